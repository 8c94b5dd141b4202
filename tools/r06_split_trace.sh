R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06so}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pbs_generic.py -q --timeout 300 --timeout-method thread > $O/pytest_generic.log 2>&1; rc=$?; tail -2 $O/pytest_generic.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
for C in "opt9 1024" "opt10 512"; do set -- $C
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$1 -o run -- python3 $R/bench.py --config $1 --batch $2 --steps 2 --warmup 1 --no-cpu-baseline --verify 0 --no-ks --no-e2e --no-sdfg --no-share > $O/trace_$1.log 2>&1 || exit 1
  grep '^{' $O/trace_$1.log | cut -c1-120
done
