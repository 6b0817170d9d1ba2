#!/bin/bash
# SQ counters of one kernel launched alone (tools/prof_zzt.py --kernel $KERNEL), in
# three rocprofv3 --pmc passes (<= 8 SQ + 2 GRBM counters each), then a JSON summary:
#   KERNEL=zzt_dense TAG=v4 bash tools/pmc_sq.sh   -> gpurun_out/pmc_$TAG.json
# (CMD overrides the launcher, e.g. CMD="python tools/ab_fast.py --keys dec:fwd --reps 2"
#  KERNEL=dec_fwd_kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
K=${KERNEL:-zzt_dense}; T=${TAG:-$K}
mkdir -p gpurun_out/pmc_$T
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_EXP SQ_INSTS_BRANCH SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmc_$T/p$i -o run --output-format csv -- \
    ${CMD:-python tools/prof_zzt.py --reps 3 --kernel $K} > gpurun_out/pmc_$T/p$i.log 2>&1 || { echo "FAILED pass $i"; tail -5 gpurun_out/pmc_$T/p$i.log; exit 1; }
done
python tools/pmc_sq.py gpurun_out/pmc_$T $K > gpurun_out/pmc_$T.json && cat gpurun_out/pmc_$T.json
