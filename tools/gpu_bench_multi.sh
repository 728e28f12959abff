set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== bench N=1" && timeout -k 10 300 python bench.py > gpurun_out/bench_n1.log 2>&1; rc=$?; tail -1 gpurun_out/bench_n1.log; [ $rc -eq 0 ] || exit $rc
echo "== bench rehearsal 2 ranks on one GPU (gloo)" && LGS_ONE_DEVICE=1 LGS_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --chains 4096 > gpurun_out/bench_n2.log 2>&1; rc=$?; tail -2 gpurun_out/bench_n2.log; exit $rc
