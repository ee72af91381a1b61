#!/bin/bash
# PMC passes of tools/xlat_probe.py: address-translation and memory-side write
# stall counters on each footprint shape, one counter group per rocprofv3 run, no trace domains.
# Output: gpurun_out/xlat/<case>_<pass>/ (CSV) + <case>_time.json (unprofiled timing).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/xlat"
mkdir -p "$O"
CASES=${CASES:-"t10 t4same t4of10 t10alt"}
declare -A P
P[tlb]="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
P[ea]="TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_TAG_STALL_sum GRBM_EA_BUSY GRBM_TC_BUSY"
P[tlb2]="TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_SERIALIZATION_STALL_sum"
P[tcp]="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_CLIENT_UTCL1_INFLIGHT_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
PASSES=${PASSES:-"tlb ea tlb2 tcp"}
cd /tmp && export TMPDIR=/tmp
for c in $CASES; do
  timeout -k 10 120 python3 "$R/tools/xlat_probe.py" $c ${PROBE_ARGS:-} > "$O/${c}_time.json" 2> "$O/${c}_time.err" || { echo "time $c rc=$?"; exit 1; }
  cat "$O/${c}_time.json"
done
for c in $CASES; do
  for p in $PASSES; do
    timeout -s KILL 90 rocprofv3 --pmc ${P[$p]} --output-format csv -d "$O/${c}_$p" -o pmc \
      -- python3 "$R/tools/xlat_probe.py" $c --launches 12 ${PROBE_ARGS:-} > "$O/${c}_$p.log" 2>&1
    rc=$?; echo "pmc $c $p rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$O/${c}_$p.log"; exit $rc; }
  done
done
python3 "$R/tools/xlat_summary.py" "$O" > "$O/summary.txt" 2>&1; cat "$O/summary.txt"
