#!/usr/bin/env bash
# PMC of the fused SwiGLU-backward dgrad against the plain dgrad of the same
# shape (scripts/gpu/swiglu_dgrad_time.py), one counter group per pass.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
O=$R/gpurun_out/swpmc
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/pmc$i -o run -- \
    python3 $R/scripts/gpu/swiglu_dgrad_time.py > $O/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/scripts/pmc_summary.py $O/pmc1 $O/pmc2 $O/pmc3 --filter x2_kernel > $O/summary.txt 2>&1
cat $O/summary.txt
