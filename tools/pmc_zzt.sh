# SQ counters of the fused zz^T + CE kernel (tools/prof_zzt.py), two per rocprofv3 pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pz
i=0
for pair in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "SQ_INSTS_LDS SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -k 5 90 rocprofv3 --pmc $pair -d gpurun_out/pz/p$i -o run --output-format csv -- python tools/prof_zzt.py --reps 3 > gpurun_out/pz/p$i.log 2>&1 || { echo "FAILED $pair"; exit 1; }
done
echo done
