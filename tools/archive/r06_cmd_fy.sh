export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CONCRETE_HIP_LIB=$R/variants/libconcrete_hip_fusey.so CONCRETE_HIP_GEN_FUSEDY=1 CONCRETE_HIP_GEN_STREAMS=1 PMC_TIMEOUT=240 \
  timeout -k 10 600 bash tools/pmc.sh r06fy/pmc_fy1 de --config opt8 --no-ks --no-sdfg --batch 1024 > gpurun_out/r06fy_pmc.log 2>&1 && echo pmc fused ok &&
bash tools/r06.sh r06j keybound
