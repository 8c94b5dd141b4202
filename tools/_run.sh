set -e -o pipefail
TAG=${1:-x}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_runtime.py -x -q > $O/pytest_rt.log 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -q > $O/pytest.log 2>&1
echo done
