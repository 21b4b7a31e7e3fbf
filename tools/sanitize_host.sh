#!/bin/bash
# The host library and the host side of libmrt.so under AddressSanitizer + UBSan
# (make sanitize -> lib-asan/), driven by the CPU tests that exercise them: the
# SBVH builder (threads), OBJ parser, .dat loader, camera decoder, wide-node
# derivation and the C-ABI's argument checks. Writes profiles/<tag>_sanitize_host.log.
#   tools/sanitize_host.sh [tag]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
TAG=${1:-round3}
make -C gpu-ray-tracing_amd -j8 sanitize > /dev/null || exit 1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
LOG=profiles/${TAG}_sanitize_host.log
{
  echo "# $(date -u +%F) host-code ASan+UBSan: make -C gpu-ray-tracing_amd sanitize (lib-asan/),"
  echo "# LD_PRELOAD=$RT, ASAN_OPTIONS=detect_leaks=0 (CPython's own allocations), UBSAN halt_on_error"
  echo "# tests: test_oracle test_bvhcache test_camera test_wide_nodes test_abi test_renderer (CPU part)"
} > $LOG
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib-asan \
  python -m pytest tests/test_oracle.py tests/test_bvhcache.py tests/test_camera.py tests/test_wide_nodes.py \
  tests/test_abi.py tests/test_renderer.py -m "not gpu" -q -p no:cacheprovider >> $LOG 2>&1
rc=$?
echo "# exit $rc" >> $LOG
grep -c "ERROR: AddressSanitizer\|runtime error:" $LOG | sed 's/^/# sanitizer reports: /' >> $LOG
tail -4 $LOG
exit $rc
