#!/bin/bash
# Round 6 closing run on the GPU box: general-path PMC records (written into profiles/ on the box so the
# bench lines that follow use them, and copied to gpurun_out/TAG/records), their bench lines, the whole
# GPU suite, smoke, the default bench and its rocprofv3 summary.  Usage: tools/r06_final.sh TAG
TAG=${1:-r06z}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O/records; cd $R
bash tools/r06.sh $TAG genprof || exit 1
for c in "opt6 4096" "opt7 1024" "opt8 1024" "opt9 128" "opt10 64"; do
  set -- $c
  python tools/pmc_record.py gpurun_out/$TAG/$1 profiles/r06_$1_pmc.json $1 $2 > /dev/null || exit 1
  cp profiles/r06_$1_pmc.json $O/records/ && cp gpurun_out/$TAG/trace_$1/run_kernel_stats.csv $O/records/r06_$1_kernel_stats.csv
done
echo "records written"
bash tools/r06.sh r06m bench3 || exit 1
bash tools/r06.sh $TAG suite || exit 1
bash tools/r06_prof_default.sh $TAG || exit 1
