# round 6 final build (df598d39): the 8-GPU command rehearsed with 2 ranks on one GPU (gloo), C4 (2^15 chains
# x 256 IMHK steps per rank per call, as BASELINE configs[3] runs per GPU); per-rank memory in the line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
LGS_ONE_DEVICE=1 LGS_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --config C4_qary1024 --steps 2 --warmup 1 > gpurun_out/r06ar_bench_2ranks_1gpu_C4.log 2>&1; rc=$?
tail -n 1 gpurun_out/r06ar_bench_2ranks_1gpu_C4.log | cut -c1-1500
exit $rc
