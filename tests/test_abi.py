"""The C-ABI libraries load and export every symbol their headers declare
(CPU-only: no kernel is launched)."""
import ctypes as C
import os
import re

import pytest

from mrt import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header):
    text = open(os.path.join(REPO, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", text)
    skip = {"if", "defined", "sizeof"}
    return sorted({n for n in names if n not in skip and not n.isupper()})


@pytest.mark.parametrize("header,path", [("mrt.h", _lib.TRACE_LIB_PATH), ("mrt_host.h", _lib.HOST_LIB_PATH)])
def test_every_declared_symbol_is_exported(header, path):
    lib = C.CDLL(path)
    names = declared_functions(header)
    assert len(names) > 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"{os.path.basename(path)} lacks {missing}"


@pytest.mark.parametrize("header,table", [("mrt.h", _lib.TRACE_SYMBOLS), ("mrt_host.h", _lib.HOST_SYMBOLS)])
def test_python_bindings_cover_the_header(header, table):
    assert sorted(n for n, _, _ in table) == declared_functions(header)


def test_reference_compat_names_present():
    # CudaTracerKernels.hh:44-52
    lib = _lib.trace_lib()
    for n in ("bind_CudaBVHTexture", "unbind_CudaBVHTexture", "launch_tracingKernel", "copy_tracing_results"):
        assert hasattr(lib, n)


def test_error_strings_and_version():
    lib = _lib.trace_lib()
    assert lib.mrt_version() >= 100
    assert lib.mrt_error_string(0) == b"ok"
    assert lib.mrt_error_string(2) == b"no BVH bound"


def test_invalid_arguments_rejected_without_gpu():
    lib = _lib.trace_lib()
    out = C.c_void_p()
    assert lib.mrt_tracer_create(0, None) == 1           # null out pointer
    rc = lib.mrt_tracer_create(0, C.byref(out))
    if lib.mrt_device_count() == 0:
        assert rc == 4                                   # MRT_ERR_NO_DEVICE
        assert out.value is None
    else:
        assert rc == 0
        lib.mrt_tracer_destroy(out)
    assert lib.mrt_tracer_trace(None, None, None, 1, 0, None, None) == 1
    assert lib.mrt_tracer_bind(None, None, 0, None, 0, None, 0) == 1


@pytest.mark.parametrize("struct,cls", [("mrt_launch_cfg", _lib.LaunchCfg), ("mrt_trace_info", _lib.TraceInfo)])
def test_ctypes_structs_match_the_header(struct, cls):
    """The Python mirrors of the C structs list the header's fields, in order."""
    text = open(os.path.join(REPO, "include", "mrt.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    body = re.search(r"typedef struct " + struct + r"\s*\{(.*?)\}\s*" + struct + ";", text, flags=re.S).group(1)
    fields = re.findall(r"\b(?:int32_t|float)\s+([A-Za-z_][A-Za-z0-9_]*)\s*;", body)
    assert fields == [n for n, _ in cls._fields_]


def test_cpp_dropin_resolves_the_reference_prototypes_from_libmrt():
    """tests/cpp/cuda_tracer_dropin.cpp declares CudaTracerKernels.hh:42-52 with the
    reference's own parameter types; its undefined symbols are exactly those four
    names (C linkage, no mangling) and libmrt.so resolves them at load time."""
    import subprocess
    exe = os.path.join(REPO, "gpu-ray-tracing_amd", "lib", "cuda_tracer_dropin")
    if not os.path.exists(exe):
        pytest.skip("not built (make -C gpu-ray-tracing_amd)")
    undef = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    wanted = {"bind_CudaBVHTexture", "unbind_CudaBVHTexture", "launch_tracingKernel", "copy_tracing_results"}
    assert wanted <= set(line.split()[-1] for line in undef.splitlines() if line.strip())
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True, check=True).stdout
    assert "libmrt.so" in ldd and "not found" not in ldd.split("libmrt.so", 1)[1].splitlines()[0]


def test_trace_flags_match_the_header():
    """The Python flag constants are the header's enum values (MRT_TRACE_SECONDARY, round 5, included)."""
    text = open(os.path.join(REPO, "include", "mrt.h")).read()
    for name in ("MRT_TRACE_ANY_HIT", "MRT_TRACE_EXACT_RCP", "MRT_TRACE_LOCKSTEP_OFF", "MRT_TRACE_STATS",
                 "MRT_TRACE_SECONDARY"):
        m = re.search(name + r"\s*=\s*1u\s*<<\s*(\d+)", text)
        assert m, name
        assert getattr(_lib, name) == 1 << int(m.group(1)), name


def test_secondary_hint_travels_with_the_buffer():
    """RayBuffer.secondary reaches the trace flags and survives view() (no GPU needed)."""
    import torch
    from mrt.tracer import RayBuffer, Tracer
    cpu = torch.device("cpu")
    rb = RayBuffer(torch.zeros((8, 8)), need_closest_hit=True, device=cpu, secondary=True)
    assert rb.view(2, 5).secondary
    assert Tracer.flags(None, rb) & _lib.MRT_TRACE_SECONDARY
    assert not Tracer.flags(None, RayBuffer(torch.zeros((8, 8)), device=cpu)) & _lib.MRT_TRACE_SECONDARY


def test_shard_blocks_size_query_and_argument_checks():
    """mrt_shard_blocks / mrt_raygen_ao_blocks host-side contract (no device needed): the
    block/ray counts of a rank's shard come back without touching the device (blocks NULL),
    including the frame's partial last block; bad arguments are refused before any launch."""
    import ctypes as C
    from mrt import _lib
    lib = _lib.trace_lib()
    n, m = C.c_int32(0), C.c_int64(0)
    # 1920x1080 at 8 spp in 1024-ray blocks: 16 200 blocks, 2 025 per rank of 8
    assert lib.mrt_shard_blocks(None, 1920 * 1080, 8, 1024, 8, 3, 1, None, 0, C.byref(n), C.byref(m), None) == 0
    assert (n.value, m.value) == (2025, 2025 * 1024)
    # 97x61 primaries x 3 samples = 17 751 rays in 128-ray blocks: 139 blocks, the last 87 rays long
    for rank, blocks in ((0, 70), (1, 69)):
        assert lib.mrt_shard_blocks(None, 97 * 61, 3, 128, 2, rank, 0, None, 0, C.byref(n), C.byref(m), None) == 0
        assert n.value == blocks
        assert m.value == blocks * 128 - (128 - 17751 % 128 if rank == 0 else 0)
    for bad in ((100, 1, 64, 0, 0, 1), (100, 1, 64, 2, 2, 1), (100, 0, 64, 1, 0, 1), (100, 1, 0, 1, 0, 1),
                (100, 1, 64, 1, 0, 2), (-1, 1, 64, 1, 0, 1)):
        np_, s, b, w, r, o = bad
        assert lib.mrt_shard_blocks(None, np_, s, b, w, r, o, None, 0, C.byref(n), C.byref(m), None) == _lib.MRT_ERR_INVALID_ARG
    # a capacity below the shard's blocks, and a live-first order over more than 16 384 blocks per rank
    dummy = C.c_void_p(1)
    assert lib.mrt_shard_blocks(dummy, 1000, 1, 64, 1, 0, 0, dummy, 3, C.byref(n), C.byref(m), None) == 5
    assert lib.mrt_shard_blocks(dummy, 1 << 20, 8, 256, 1, 0, 1, dummy, 1 << 20, C.byref(n), C.byref(m), None) == 5
    seeds = (C.c_uint32 * 1)(1804289383)
    sp = C.cast(seeds, C.c_void_p)
    # nothing listed: no launch; more blocks listed than the frame has, or a wrong ray count: refused
    assert lib.mrt_raygen_ao_blocks(None, None, 100, None, 0, 2, 5.0, sp, 1, 1000, None, 0, 64, 0, None, None) == 0
    assert lib.mrt_raygen_ao_blocks(dummy, dummy, 100, None, 0, 2, 5.0, sp, 1, 1000, dummy, 5, 64, 5 * 64,
                                    dummy, None) == _lib.MRT_ERR_INVALID_ARG
    assert lib.mrt_raygen_ao_blocks(dummy, dummy, 100, None, 0, 2, 5.0, sp, 1, 1000, dummy, 2, 64, 2 * 64 + 1,
                                    dummy, None) == _lib.MRT_ERR_INVALID_ARG
    # fewer seeds than the frame's batches (100 inputs at 30 per batch: 4 batches)
    assert lib.mrt_raygen_ao_blocks(dummy, dummy, 100, None, 0, 2, 5.0, sp, 1, 30, dummy, 1, 64, 64,
                                    dummy, None) == _lib.MRT_ERR_INVALID_ARG
