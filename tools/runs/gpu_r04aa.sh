# multi-rank rehearsal on one GPU (gloo; the driver's 8-GPU node uses RCCL): the
# self-launching bench at 2 ranks (C3) and 4 ranks (C4, the 8-GPU config's shape)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export LGS_ONE_DEVICE=1 LGS_DIST_BACKEND=gloo
echo "== 2 ranks C3" && timeout -k 10 400 python bench.py --gpus 2 --no-cpu --steps 3 --warmup 1 > gpurun_out/r04aa_2.log 2>&1; rc=$?; tail -1 gpurun_out/r04aa_2.log | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04aa_2.log; exit $rc; }
echo "== 4 ranks C4" && timeout -k 10 500 python bench.py --gpus 4 --config C4_qary1024 --no-cpu --steps 3 --warmup 1 > gpurun_out/r04aa_4.log 2>&1; rc=$?; tail -1 gpurun_out/r04aa_4.log | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04aa_4.log; exit $rc; }
