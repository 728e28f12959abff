# round 6: PC sampling of the Klein kernel (C3, 2^18 samples) -- where the waves' time goes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
echo "== stochastic"
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d gpurun_out/pcs/st -o st --output-format csv -- python3 tools/kbench.py --one --config C3_ntru512 --n 262144 --reps 2 > gpurun_out/pcs/st.log 2>&1; rc=$?
echo "rc=$rc"; tail -5 gpurun_out/pcs/st.log
if [ $rc -ne 0 ] && [ $rc -ne 124 ] && [ $rc -ne 137 ]; then
  echo "== host_trap"
  timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 -d gpurun_out/pcs/ht -o ht --output-format csv -- python3 tools/kbench.py --one --config C3_ntru512 --n 262144 --reps 2 > gpurun_out/pcs/ht.log 2>&1; rc=$?
  echo "rc=$rc"; tail -5 gpurun_out/pcs/ht.log
fi
find gpurun_out/pcs -type f | head -20
exit 0
