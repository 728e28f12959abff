# Profile of the bench command for bench.py's roofline: rocprofv3 kernel trace +
# --stats, then separate --pmc passes (SQ instruction mix, issue/wait, FETCH_SIZE,
# WRITE_SIZE) under gpurun_out/prof_TAG; then, in the container, summarise into
# profiles/: python3 tools/summarize_prof.py gpurun_out/prof_TAG TAG and
# python3 tools/roofline_counters.py gpurun_out/prof_TAG CFG UNITS D profiles/TAG_klein_counters.json
# usage: bash tools/gpu_roofline.sh TAG [config]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
CFG=${2:-C3_ntru512}
ARGS="--steps 3 --warmup 1 --no-cpu --wl-steps 0 --config $CFG"
# Isolated launches (round 5): the bench pipelines each block's Klein launch beside the
# previous block's B z; under rocprofv3 that overlap changes (the profiled bench ran at
# 93.8 instead of 105 M samples/s, its Klein launches stretched to 10.0 ms by both
# clocks, profiles/r05x_*), so the counters and the kernel's duration come from the
# same command with LGS_NO_PIPE=1, where each launch has the chip to itself
# (PROF_NO_PIPE=0: profile the pipelined command)
export LGS_NO_PIPE=${PROF_NO_PIPE:-1}
O=gpurun_out/prof_$TAG
mkdir -p $O profiles
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS > $O/bench_trace.log 2>&1 || { tail -20 $O/bench_trace.log; exit 1; }
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
i=0
for P in "sq1:$P1" "sq2:$P2" "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
  name=${P%%:*}
  timeout -s KILL 300 rocprofv3 --pmc ${P#*:} -d $O/pmc_$name -o run --output-format csv -- python3 bench.py $ARGS > $O/bench_pmc_$name.log 2>&1 || { echo "pmc pass $name failed"; tail -20 $O/bench_pmc_$name.log; exit 1; }
done
D=$(python3 -c "import sys; sys.path.insert(0,'lattice-gaussian-mcmc_amd'); from lgs_amd.lattices import build_config; print(build_config('$CFG')[0].basis.shape[0])")
UNITS=$(python3 -c "import json; l=[x for x in open('$O/bench_trace.log') if x.startswith('{')][-1]; print(json.loads(l)['roofline']['units_per_launch'])")
python3 tools/co_resources.py --filter _ZN3lgs --json $O/${TAG}_co_resources.json > $O/co_resources.txt
python3 tools/roofline_counters.py $O $CFG $UNITS $D $O/${TAG}_klein_counters.json $O/bench_trace.log $O/${TAG}_co_resources.json
