#!/bin/bash
# Lists the box's counters (rocprofv3 -L) and runs ONE --pmc pass of the C2
# (or $1) path kernel with the candidates below that the list knows (at most
# 8 SQ-block counters, 2 GRBM: one pass).  Output under gpurun_out/$TAG.
#   gpurun -- bash tools/pmc_probe.sh <tag> [workload] [counters...]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-probe}; W=${2:-C2}; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
CANDS=${*:-"SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY"}
SEL=""
for c in $CANDS; do
  if grep -qw "$c" "$OUT/counters.txt"; then SEL="$SEL $c"; else echo "not listed: $c"; fi
done
echo "pass:$SEL"
[ -n "$SEL" ] || exit 0
timeout -k 10 300 rocprofv3 --pmc $SEL --output-format csv -d "$OUT/pmc" -o run \
  -- python3 bench.py --workload "$W" --steps 1 --warmup 0 --no-cpu-baseline --no-pmc > "$OUT/pmc.log" 2>&1
rc=$?
echo "pmc rc=$rc"; tail -2 "$OUT/pmc.log"
[ $rc -eq 0 ] && python3 tools/pmc_summary.py "$OUT/pmc" | tee "$OUT/summary.txt"
exit $rc
