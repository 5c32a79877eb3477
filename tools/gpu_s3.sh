set -o pipefail
O=gpurun_out/s3
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 &&
bash tools/prof.sh $O/prof --steps 10 --no-cpu-baseline
