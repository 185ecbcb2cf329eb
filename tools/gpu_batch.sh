#!/bin/bash
# One gpurun batch: GPU parity tests, C3 bench, kernel-trace profile, then PMC
# passes (each counter group in its own run, no trace domains besides the
# kernel dispatches).  Every GPU step has its own time limit and the chain stops
# at the first failure.
#   gpurun --timeout 1200 -- bash tools/gpu_batch.sh <tag> [steps...]
# steps: tests bench c2 c3 c5 prof2 prof3 pmc2 pmc3 occ2 mix2 eff2 ... (default: the list below)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-run}; shift
STEPS=${*:-"tests c3 prof3 pmc3 pmc2 occ2"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
B="python3 bench.py"
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -3 "$OUT/$name.log"
  return $rc
}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
    bench) run bench_default 900 $B --gpus 1 --steps 20 --warmup 5 || exit 1 ;;
    multi) run pytest_multi 600 python3 -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 300 \
             --timeout-method thread || exit 1 ;;
    dist2) # the N=2 bench path (PMC children, tile shares, one gather, max-over-ranks) as a gloo rehearsal
      run bench_dist2 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo || exit 1 ;;
    rehearse8)  # the driver's exact N=8 command, PMC passes on, all 8 gloo ranks on this one GPU
      run bench_rehearsal_gloo8_pmc 900 $B --gpus 8 --dist-backend gloo || exit 1 ;;
    wr2|wr3|wr5)  # where the writes come from: L2->fabric write requests by size, then the store
      # instruction mix (VMEM / FLAT incl. scratch) — $WR_LIB (default the product), $WR_SPP
      w=C${s#wr}
      RT_AMD_LIB=${WR_LIB:-$PWD/cpu-raytracing-rt_amd/build/librt_amd.so} run wreq_$w 600 rocprofv3 --pmc \
        TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv \
        -d "$OUT/wreq_$w" -o run -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc \
        ${WR_SPP:+--spp $WR_SPP} ${WR_TUNE:+--tune $WR_TUNE} || exit 1
      RT_AMD_LIB=${WR_LIB:-$PWD/cpu-raytracing-rt_amd/build/librt_amd.so} run wins_$w 600 rocprofv3 --pmc \
        SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_FLAT \
        TCP_TCC_WRITE_REQ_sum --output-format csv -d "$OUT/wins_$w" -o run \
        -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc ${WR_SPP:+--spp $WR_SPP} \
        ${WR_TUNE:+--tune $WR_TUNE} || exit 1 ;;
    hit3|hit5)  # L1 (TCP) and L2 (TCC) hit rates of the path kernel's loads, with --tune $TUNE
      w=C${s#hit}
      run tcphit_${w}_$(echo "$TUNE" | tr ',=' '__') 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum \
        TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv \
        -d "$OUT/tcphit_${w}_$(echo "$TUNE" | tr ',=' '__')" -o run -- $B --workload $w --steps 1 --warmup 0 \
        --no-cpu-baseline --no-pmc --spp ${HIT_SPP:-16} --tune "$TUNE" || exit 1 ;;
    tc3|tc5)  # the full-frame bench of C3 / C5 with --tune $TUNE (a kernel form the host does not pick yet)
      w=C${s#tc}
      run bench_${w}_$(echo "$TUNE" | tr ',=' '__') 900 $B --workload $w --steps 2 --warmup 1 --tune "$TUNE" || exit 1 ;;
    c2)    run bench_c2 600 $B --workload C2 --steps 3 --warmup 1 || exit 1 ;;
    c3)    run bench_c3 600 $B --workload C3 --steps 3 --warmup 1 || exit 1 ;;
    c5)    run bench_c5 900 $B --workload C5 --steps 2 --warmup 1 || exit 1 ;;
    prof2) run prof_c2 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o run \
             -- $B --workload C2 --steps 2 --warmup 1 --no-cpu-baseline --no-pmc || exit 1 ;;
    prof3) run prof_c3 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o run \
             -- $B --workload C3 --steps 2 --warmup 1 --no-cpu-baseline --no-pmc || exit 1 ;;
    prof5) run prof_c5 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run \
             -- $B --workload C5 --steps 2 --warmup 1 --no-cpu-baseline --no-pmc || exit 1 ;;
    pmc2|pmc3)
      w=C${s#pmc}
      run fetch_$w 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$w" -o run \
        -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc || exit 1
      run write_$w 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_$w" -o run \
        -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc || exit 1 ;;
    occ2)  run occ_C2 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
             --output-format csv -d "$OUT/occ_C2" -o run \
             -- $B --workload C2 --steps 1 --warmup 0 --no-cpu-baseline --no-pmc || exit 1 ;;
    ctrs)  run counters 300 rocprofv3 -L || exit 1 ;;
    mix2|mix3)  # SQ instruction mix + stall cycles of the path kernel (one SQ pass, 8 slots)
      w=C${s#mix}
      run mix_$w 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
        SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d "$OUT/mix_$w" -o run \
        -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc || exit 1 ;;
    eff2|eff3)  # lane efficiency + f64/int mix (SQ pass), then L2 hit rate + L1->L2 latency (TCC/TCP pass)
      w=C${s#eff}
      run eff_$w 600 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 \
        SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 \
        --output-format csv -d "$OUT/eff_$w" -o run \
        -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc || exit 1
      run l2_$w 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum \
        --output-format csv -d "$OUT/l2_$w" -o run \
        -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc || exit 1 ;;
    phase2|phase3|phase5)  # per-region wave cycles from the -DRT_PHASES build (cpu-raytracing-rt_amd/ph_build)
      w=C${s#phase}
      RT_AMD_LIB=$PWD/cpu-raytracing-rt_amd/ph_build/librt_amd.so run phase_$w 600 \
        python3 tools/phases.py $w ${PHASE_SPP:-64} || exit 1 ;;
    lane2) run lane_C2 600 python3 tools/lane_util.py C2 256 256 64 32 8 || exit 1 ;;
    lane3) run lane_C3 600 python3 tools/lane_util.py C3 64 64 32 8 || exit 1 ;;
    var2|var3)  # every cpu-raytracing-rt_amd/build*/librt_amd.so variant at reduced spp
      w=C${s#var}
      run variants_$w 900 python3 tools/variants.py $w ${VAR_SPP:-64} ${VARIANTS:-cpu-raytracing-rt_amd/build*/librt_amd.so} \
        || exit 1 ;;
    wait2|wait3|wait5)  # where wave-time goes: parked on s_waitcnt vs issue stalls vs issuing (one SQ pass)
      w=C${s#wait}
      run wait_$w 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
        SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --output-format csv -d "$OUT/wait_$w" -o run \
        -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc ${WAIT_SPP:+--spp $WAIT_SPP} || exit 1 ;;
    l1_2|l1_3|l1_5)  # vector-memory pipe: TA/TD busy and stalls, then L1 (TCP) stalls and latency
      w=C${s#l1_}
      run ta_$w 600 rocprofv3 --pmc TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum \
        GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/ta_$w" -o run \
        -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc ${WAIT_SPP:+--spp $WAIT_SPP} || exit 1
      run tcp_$w 600 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_LATENCY_sum \
        TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d "$OUT/tcp_$w" -o run \
        -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc ${WAIT_SPP:+--spp $WAIT_SPP} || exit 1 ;;
    share2) run share_C2 600 python3 tools/share_scaling.py C2 256 1 8 || exit 1 ;;
    share4) run share_C4 900 python3 tools/share_scaling.py C4 1024 1 8 || exit 1 ;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    c4)    run bench_c4 900 $B --workload C4 --steps 2 --warmup 1 || exit 1 ;;
    prof4) run prof_c4 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run \
             -- $B --workload C4 --steps 2 --warmup 1 --no-cpu-baseline --no-pmc || exit 1 ;;
    prof5) run prof_c5 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run \
             -- $B --workload C5 --steps 2 --warmup 1 --no-cpu-baseline --no-pmc || exit 1 ;;
    var5)  run variants_C5 900 python3 tools/variants.py C5 ${VAR_SPP5:-16} \
             ${VARIANTS:-cpu-raytracing-rt_amd/build*/librt_amd.so} || exit 1 ;;
    calib)  # FETCH_SIZE / TCC_EA0_RDREQ* factors for the traversal's record gathers (tools/fetch_calib.hip)
      run calib_plain 120 tools/fetch_calib || exit 1
      run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o run \
        -- tools/fetch_calib || exit 1
      run calib_rdreq 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
        TCC_EA0_RDREQ_128B_sum --output-format csv -d "$OUT/calib_rdreq" -o run -- tools/fetch_calib || exit 1
      run calib_dram 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum --output-format csv \
        -d "$OUT/calib_dram" -o run -- tools/fetch_calib || exit 1
      run calib_report 60 python3 tools/fetch_calib.py "$OUT" || exit 1 ;;
    c5t)   run pytest_c5 900 python3 -u -m pytest tests/test_gpu_c5.py -m gpu -x -v --timeout 600 \
             --timeout-method thread || exit 1 ;;
    kids)  run kid_stats 600 python3 tools/kid_stats.py C3 64 C5 16 || exit 1 ;;
    valu)  run valu_rates 300 tools/valu_rates full || exit 1 ;;
    lanes2|lanes3)  # active lanes per VALU instruction of a variant library ($LANES_LIB, default the product)
      w=C${s#lanes}
      RT_AMD_LIB=${LANES_LIB:-$PWD/cpu-raytracing-rt_amd/build/librt_amd.so} run lanes_$w 600 rocprofv3 --pmc \
        SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d "$OUT/lanes_$w" \
        -o run -- $B --workload $w --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --spp ${LANES_SPP:-64} || exit 1 ;;
    sortpmc)  # the one-wave and the regrouped C2 kernels side by side: instruction mix, lanes, waits, LDS
      for tn in sorted=0 sorted=1; do
        run sq_$tn 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
          SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d "$OUT/sq_$tn" -o run \
          -- $B --workload C2 --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --spp 64 --tune $tn || exit 1
        run lds_$tn 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY \
          SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --output-format csv -d "$OUT/lds_$tn" -o run \
          -- $B --workload C2 --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --spp 64 --tune $tn || exit 1
      done ;;
    *)     echo "unknown step $s"; exit 2 ;;
  esac
done
echo "[$(date +%T)] batch done"
