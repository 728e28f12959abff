# round-4 consolidated GPU call: new tests, q-skip A/B, full suite, bench, B z
# variants, roofline profile (trace + PMC passes) of the bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r04d}
echo "== new tests" && timeout -k 10 500 python -u -m pytest tests/test_gpu_wl_accept.py tests/test_gpu_certificate.py tests/test_gpu_stream.py -x -v -s --timeout 300 --timeout-method thread -k "wl_accept or speculative or q_panel or functionals or streams" > gpurun_out/${T}_new.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|scale|bounds|differ|passed|failed|skip |assert" gpurun_out/${T}_new.log | tail -40; [ $rc -eq 0 ] || exit $rc
echo "== kbench qskip A/B" && for q in 1 0 1 0; do LGS_NO_QSKIP=$q timeout -k 10 120 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash --bz || exit 1; done > gpurun_out/${T}_kbench.log 2>&1; rc=$?; cat gpurun_out/${T}_kbench.log | tail -4; [ $rc -eq 0 ] || exit $rc
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bench.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
echo "== bz variants" && LGS_LIBS=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:lattice-gaussian-mcmc_amd/build/var/noclive.so:lattice-gaussian-mcmc_amd/build/var/bznomfma.so:lattice-gaussian-mcmc_amd/build/var/bznostore.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --bz > gpurun_out/${T}_bzvar.log 2>&1; rc=$?; cat gpurun_out/${T}_bzvar.log | tail -4; [ $rc -eq 0 ] || exit $rc
echo "== roofline profile" && timeout -k 10 900 bash tools/gpu_roofline.sh $T > gpurun_out/${T}_roof.log 2>&1; rc=$?; tail -5 gpurun_out/${T}_roof.log; exit $rc
