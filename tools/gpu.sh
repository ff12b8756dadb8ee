#!/bin/bash
# The one GPU-box driver (replaces round 1-2's one-off tools/gpu_*.sh A/B scripts). Libraries are prebuilt in-tree
# on the CPU container; nothing is compiled here.
#
#   TAG=name bash tools/gpu.sh STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failing step ends the call (no retries).
#   tests[:K_EXPR]            pytest -m gpu [-k K_EXPR]                         -> tests.log
#   smoke                     __graft_entry__.smoke()                           -> smoke.log
#   bench:GAME[:ARGS...]      python bench.py --game GAME ARGS (ARGS ','-separated) -> bench_GAME.jsonl
#   counters:GAME:N:T         SQ instruction / wait counters over tools/ab_rollout.py, one PMC pass per group
#   profile:GAME[:ARGS...]    kernel trace + stats, then FETCH_SIZE and WRITE_SIZE passes over bench.py
#   ab:GAME:N:T:F1[:F2...]    tools/ab_rollout.py kernel-flag A/B (AB_PLAYERS / AB_WARM from the env)
#   abl:GAME:N:T:LIB1[:LIB2]  the same rollout timed with several library builds (CARDSIM_LIB), interleaved runs
#   abx:GAME:N:T:LIB1[:LIB2]  the same, all libraries in one process writing the same trajectory buffers
#   devstate / listctr        device state (tools/device_state.py), rocprofv3 -L
#   pmc:GAME:N:T:CTR...       one PMC pass over tools/ab_rollout.py
#   ceiling                   plain read / write streams and torch fill_ on this box (tools/calib.py --ceiling)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
O=$R/gpurun_out/${TAG:-run}
mkdir -p "$O"
echo "host $(hostname) $(date -u +%FT%TZ) head $(cat .git_head 2>/dev/null)" >> "$O/steps.log"

run() {   # run LIMIT LOG cmd...
  local lim=$1 log=$2; shift 2
  echo "[$(date -u +%T)] $*" >> "$O/steps.log"
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$(date -u +%T)] rc=$rc" >> "$O/steps.log"
  if [ $rc -ne 0 ]; then tail -30 "$log"; exit $rc; fi
}

for step in "$@"; do
  IFS=':' read -r -a a <<< "$step"
  case "${a[0]}" in
    tests)
      if [ -n "${a[1]}" ]; then
        run 900 "$O/tests.log" python3 -u -m pytest tests -m gpu --maxfail=15 -v --timeout 300 --timeout-method thread -k "${a[1]}"
      else
        run 1000 "$O/tests.log" python3 -u -m pytest tests -m gpu --maxfail=15 -v --timeout 300 --timeout-method thread
      fi
      tail -3 "$O/tests.log" ;;
    smoke)
      run 300 "$O/smoke.log" python3 -c "import __graft_entry__ as g; g.smoke()"
      tail -6 "$O/smoke.log" ;;
    bench)
      g=${a[1]}; extra=$(echo "${a[*]:2}" | tr ',' ' ')
      run 400 "$O/bench_$g.err" python3 bench.py --game "$g" $extra
      grep '^{' "$O/bench_$g.err" > "$O/bench_$g.jsonl"; cat "$O/bench_$g.jsonl" ;;
    counters)
      g=${a[1]}; n=${a[2]}; t=${a[3]}; d=$O/cnt_$g; mkdir -p "$d"; i=0
      for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
                 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" \
                 "FETCH_SIZE" "WRITE_SIZE" \
                 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"; do
        i=$((i+1))
        run 240 "$d/run$i.log" rocprofv3 --pmc $grp --output-format csv -d "$d/p$i" -o p -- python3 tools/ab_rollout.py "$g" "$n" "$t" 0
      done
      python3 tools/pmc_summary.py "$d" > "$d/summary.txt" 2>&1; cat "$d/summary.txt" ;;
    profile)
      g=${a[1]}; extra=$(echo "${a[*]:2}" | tr ',' ' '); d=$O/prof_$g; mkdir -p "$d"
      B="bench.py --game $g --no-cpu-baseline --no-philox --no-device-state --placement 0 --gather none --steps ${STEPS:-100} $extra"   # no amd-smi child: under rocprofv3 its env -> python3 hop is an exec after GPU init
      run 300 "$d/bench_kt.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$d/kt" -o kt -- python3 $B
      run 300 "$d/bench_fetch.log" rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$d/fetch" -o fetch -- python3 $B
      run 300 "$d/bench_write.log" rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$d/write" -o write -- python3 $B
      grep '^{' "$d/bench_kt.log" | tail -1 ;;
    vcnt)   # vcnt:GAME:N:T:LIB1[:LIB2..]  instruction counts of k_rollout per library build (one PMC pass each)
      g=${a[1]}; n=${a[2]}; t=${a[3]}; d=$O/vcnt_$g; mkdir -p "$d"
      for lib in "${a[@]:4}"; do
        CARDSIM_LIB=$lib run 240 "$d/$lib.log" rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d "$d/$lib" -o p -- python3 tools/ab_rollout.py "$g" "$n" "$t" 0
        echo "== $lib" >> "$d/summary.txt"; python3 tools/pmc_summary.py "$d/$lib" >> "$d/summary.txt" 2>&1
      done
      cat "$d/summary.txt" | grep -A 9 "== \|k_rollout" ;;
    ab)
      run 400 "$O/ab_${a[1]}.log" python3 tools/ab_rollout.py "${a[1]}" "${a[2]}" "${a[3]}" "${a[@]:4}"
      cat "$O/ab_${a[1]}.log" ;;
    abx)   # abx:GAME:N:T:LIB1[:LIB2..]  libraries A/B in ONE process over shared trajectory buffers (tools/ab_libs.py)
      run 600 "$O/abx_${a[1]}.log" python3 tools/ab_libs.py "${a[1]}" "${a[2]}" "${a[3]}" "${a[@]:4}"
      cat "$O/abx_${a[1]}.log" ;;
    pdef)   # pdef:GAME:N:T:K  default (probe-selected) vs unselected trajectory placements (tools/placement_default.py)
      run 400 "$O/pdef_${a[1]}.jsonl" python3 tools/placement_default.py "${a[1]}" "${a[2]}" "${a[3]}" "${a[4]}"
      tail -1 "$O/pdef_${a[1]}.jsonl" ;;
    abl)
      g=${a[1]}; n=${a[2]}; t=${a[3]}
      for rnd in 1 2 3; do
        for lib in "${a[@]:4}"; do
          echo "== $lib round $rnd" >> "$O/abl_$g.log"
          CARDSIM_LIB=$lib run 300 "$O/abl_tmp.log" python3 tools/ab_rollout.py "$g" "$n" "$t" 0
          sed "s|^|$lib |" "$O/abl_tmp.log" >> "$O/abl_$g.log"
        done
      done
      cat "$O/abl_$g.log" ;;
    devstate)   # the box's device state (HIP attributes + raw amd-smi metric / static / partition JSON)
      run 120 "$O/devstate.json" python3 tools/device_state.py --full
      head -c 1500 "$O/devstate.json"; echo ;;
    listctr)    # the PMC counters rocprofv3 offers on this box
      run 120 "$O/counters_avail.txt" rocprofv3 -L
      grep -i -c "" "$O/counters_avail.txt" ;;
    pmc)        # pmc:GAME:N:T:CTR1[:CTR2..]  one PMC pass (caller keeps within the per-block limits)
      g=${a[1]}; n=${a[2]}; t=${a[3]}; d=$O/pmc_${g}_$(echo "${a[@]:4}" | tr ' ' '_' | cut -c1-60); mkdir -p "$d"
      run 120 "$d/run.log" rocprofv3 --pmc ${a[@]:4} --output-format csv -d "$d/p" -o p -- python3 tools/ab_rollout.py "$g" "$n" "$t" 0
      python3 tools/pmc_summary.py "$d" > "$d/summary.txt" 2>&1; grep -A 12 k_rollout "$d/summary.txt" | head -30 ;;
    tlb)        # tlb:GAME:INST:CTR1[:CTR2..]  per-allocation k_rollout time vs counters (tools/tlb_probe.py, one PMC pass)
      g=${a[1]}; ni=${a[2]}; d=$O/tlb_${g}_$(echo "${a[@]:3}" | tr ' ' '_' | cut -c1-60); mkdir -p "$d"
      run 300 "$d/run.log" rocprofv3 --pmc ${a[@]:3} --output-format csv -d "$d/p" -o p -- python3 tools/tlb_probe.py "$g" "$ni" 6
      python3 tools/tlb_summary.py "$d" 6 > "$d/summary.txt" 2>&1; cat "$d/summary.txt"; grep instance "$d/run.log" ;;
    place)      # place:GAME:MODE:K  which allocation's placement sets the time (tools/place_probe.py)
      run 300 "$O/place_${a[1]}_${a[2]}.log" python3 tools/place_probe.py "${a[1]}" "${a[2]}" "${a[3]}"
      grep -v amdgpu.ids "$O/place_${a[1]}_${a[2]}.log" ;;
    place2)     # place2:GAME:WHAT:K  which trajectory tensor's placement matters (tools/place_probe2.py)
      run 300 "$O/place2_${a[1]}_${a[2]}.log" python3 tools/place_probe2.py "${a[1]}" "${a[2]}" "${a[3]}"
      grep -v amdgpu.ids "$O/place2_${a[1]}_${a[2]}.log" ;;
    fill)       # fill:GIB:K  plain write / read rates of K allocations (tools/fill_probe.py)
      run 300 "$O/fill_${a[1]}_${a[2]}.log" python3 tools/fill_probe.py "${a[1]}" "${a[2]}"
      grep -v amdgpu.ids "$O/fill_${a[1]}_${a[2]}.log" ;;
    tlbt)       # tlbt:GAME:INST  the same probe without a profiler (event times per allocation)
      run 300 "$O/tlbt_${a[1]}.log" python3 tools/tlb_probe.py "${a[1]}" "${a[2]}" 6
      cat "$O/tlbt_${a[1]}.log" ;;
    ceiling)
      run 300 "$O/ceiling.json" python3 tools/calib.py --ceiling
      cat "$O/ceiling.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
