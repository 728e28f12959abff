set -o pipefail
cd $GRAFT_REPO_ROOT
V=lattice-gaussian-mcmc_amd/build/var
export LGS_LIBS=$V/noinline.so:$V/inline.so
timeout -k 10 300 python tools/kbench.py --reps 3 > gpurun_out/kb32.log 2>&1 && cat gpurun_out/kb32.log &&
LGS_PANEL=16 timeout -k 10 300 python tools/kbench.py --reps 3 > gpurun_out/kb16.log 2>&1 && cat gpurun_out/kb16.log &&
LGS_LIBS=$V/noinline.so timeout -k 10 300 python tools/kbench.py --reps 1 --exact --n 65536 > gpurun_out/kbex.log 2>&1; cat gpurun_out/kbex.log
