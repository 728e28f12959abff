# round 5: Klein A/B -- Philox blocks of a quad of slots computed together (ph2), drawn
# under the record's LDS reads (ph2top), erfinv coefficients as scalar immediates
# (capimm), all three (allx); hashes must equal main's
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
echo "== kbench C3" && for r in 1 2; do LGS_LIBS=$M:$V/ph2.so:$V/ph2top.so:$V/capimm.so:$V/allx.so:$V/capbl.so:$V/disp.so:$V/tail2.so timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/r05e_kb.log
# SQ wait / issue breakdown and instruction-cache counters of main's Klein launch
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/sqpmc_r05e
mkdir -p $OUT
P3="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
P4="SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU"
P5="SQC_ICACHE_MISSES SQC_ICACHE_HITS"
for i in 3 4 5; do
  eval P=\$P$i
  echo "== pmc p$i" && LGS_LIB=$M timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/main/p$i -o run --output-format csv -- python3 $R/tools/kbench.py --one --reps 1 --n 262144 > $OUT/main.p$i.log 2>&1 || { tail -5 $OUT/main.p$i.log; echo "pass p$i failed"; }
done
python3 $R/tools/sq_summary.py $OUT klein | tee gpurun_out/r05e_sq.log
