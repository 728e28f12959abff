# SQ instruction-mix counters of the Klein kernel (kbench), per library variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$R/gpurun_out/sqpmc
mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
P3="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT64 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY"
P4="SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM"
for v in ${SQ_VARIANTS:-"main:lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so nosz:lattice-gaussian-mcmc_amd/build/var/nosz.so"}; do
  name=${v%%:*}; lib=$R/${v#*:}
  for i in ${SQ_SEL:-1 2 3 4}; do
    eval P=\$P$i
    LGS_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $P -d $OUT/$name/p$i -o run --output-format csv -- python3 $R/tools/kbench.py --one --reps 1 ${KB_ARGS} > $OUT/$name.p$i.log 2>&1 || { tail -20 $OUT/$name.p$i.log; exit 1; }
  done
done
python3 $R/tools/sq_summary.py $OUT ${SQ_KERNEL:-klein}
