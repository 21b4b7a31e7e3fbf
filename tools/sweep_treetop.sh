cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tt.log 2>&1 || { tail -30 gpurun_out/pytest_tt.log; exit 1; }
tail -2 gpurun_out/pytest_tt.log
args=()
for w in bunny-primary-1024x768 bunny-primary-640x480 conference-ao-640x480 sponza-diffuse-640x480 hairball-diffuse-640x480 hairball-diffuse-1920x1080; do
  args+=("--workload $w" "--workload $w --lds-stack 8 --treetop 320" "--workload $w --lds-stack 16 --treetop 320" "--workload $w --lds-stack 8 --treetop 128")
done
bash tools/sweep_bench.sh "${args[@]}"
