cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_latency.py -v -s -p no:cacheprovider --timeout 250 --timeout-method thread > gpurun_out/latency.log 2>&1; echo "latency rc=$?"; grep -E "passed|failed|first_call|\{" gpurun_out/latency.log | head
bash tools/prof_kernels.sh r02a --steps 100
