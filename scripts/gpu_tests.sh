set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
nproc > gpurun_out/nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -rf --timeout 600 > gpurun_out/t1.log 2>&1
