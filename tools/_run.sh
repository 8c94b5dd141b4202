set -e -o pipefail
TAG=${1:-x}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
echo done
