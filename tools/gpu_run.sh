set -e
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/t.log 2>&1
