set -uo pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4.sh r4d || exit 1
CFG=2 bash tools/ab_lib.sh r3base > gpurun_out/ab_r4d_c2.txt 2>&1 || exit 1
cat gpurun_out/ab_r4d_c2.txt
CFG=ns bash tools/ab_lib.sh r3base > gpurun_out/ab_r4d_ns.txt 2>&1 || exit 1
cat gpurun_out/ab_r4d_ns.txt
