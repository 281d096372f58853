set -o pipefail
mkdir -p gpurun_out/final2
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final2/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1 && \
timeout -k 10 240 python -u bench.py > gpurun_out/final2/bench_validator.log 2>&1 && \
timeout -k 10 400 python -u bench.py --mode ddp --steps 10 --warmup 3 > gpurun_out/final2/bench_ddp.log 2>&1
