set -e -o pipefail
TAG=${1:-x}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline > $O/bench4.log 2>&1
echo done
