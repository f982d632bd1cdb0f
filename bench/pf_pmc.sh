#!/usr/bin/env bash
# rocprofv3 PMC passes over bench/pf_pmc.py (one run per counter group; each pass under
# its own kill timeout): bash bench/pf_pmc.sh [driver args]; DRIVER (default
# bench/pf_pmc.py) picks the driver script, OUT the output directory under gpurun_out/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
o=$R/gpurun_out/${OUT:-pmc}; mkdir -p "$o"
drv=$R/${DRIVER:-bench/pf_pmc.py}
cd /tmp && export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY" \
  "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY" \
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$o/p$i" -o run -- python3 "$drv" "$@" \
      > "$o/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$o/p$i.log"; exit 1; }
  echo "pass $i ok"
done
python3 "$R/bench/pmc_summary.py" "$o"/p* > "$o/summary.md"
