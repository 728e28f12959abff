# q-skip evidence + variant A/B + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== qskip test" && timeout -k 10 300 python -u -m pytest tests/test_gpu_certificate.py -x -v -s --timeout 250 --timeout-method thread -k "q_panel" > gpurun_out/r04f_q.log 2>&1; rc=$?; grep -E "skipped|PASS|FAIL|assert|Error" gpurun_out/r04f_q.log | tail -20; [ $rc -eq 0 ] || exit $rc
V=lattice-gaussian-mcmc_amd/build/var
LIBS=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/noq.so:$V/r03.so
echo "== kbench A/B" && for r in 1 2; do LGS_LIBS=$LIBS timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --bz || exit 1; done > gpurun_out/r04f_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r04f_ab.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04f_bench.log 2>&1; rc=$?; tail -1 gpurun_out/r04f_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'])"; exit $rc
