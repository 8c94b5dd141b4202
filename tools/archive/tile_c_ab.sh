set -e -o pipefail
cd $GRAFT_REPO_ROOT
for TC in 0 2; do
  CONCRETE_HIP_TILE_C=$TC tools/opt_bench.sh tc$TC "--steps 3 --warmup 1 --no-cpu" opt1:4096 opt3:4096
done
