#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05ntt}
mkdir -p $O
cd $R/tools/microbench
timeout -k 10 120 ./ntt_bench > $O/ntt_bench.log 2>&1; rc=$?
cat $O/ntt_bench.log
[ $rc -ne 0 ] && exit $rc
cd $R
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1; rc=$?
tail -1 $O/bench_default.log | cut -c1-3000
exit $rc
