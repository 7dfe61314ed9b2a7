#!/bin/bash
# One gpurun call: the round's hardware checkpoint.  Every GPU step has its own
# time limit; a test failure (rc 1) does not stop the script, a timeout / signal /
# abort (rc >= 124) does — nothing else touches the GPU after that.
#   gpurun --timeout 1100 -- 'bash tools/gpu_check.sh <tag> [steps...]'
# steps (default: tests smoke bench): tests testsall testsx smoke bench bench2 rocprof
#   round 4: smprobe cpprobe graphcost testsnw testsdb wedge (the wedged-queue test last, alone)
set -u
TAG=${1:-r2}; shift || true
STEPS=${*:-testsall smoke bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name (limit ${lim}s) $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    bench3) run bench3 600 python -u bench.py --steps 20 --warmup 5 --pmc-lean 3 --out "$OUT/bench3.json" ;;
    train3) run train3 600 python -u bench.py --load train --steps 10 --warmup 2 --rounds 32 --hz-list 100 \
              --capacity-hz "" --burst-s 0 --quiet-s 0 --component-s 0 --pmc-lean 3 --out "$OUT/train3.json" ;;
    trainpmfw) run trainpmfw 600 python -u bench.py --load train --steps 10 --warmup 2 --rounds 32 --hz-list 100 \
              --capacity-hz "" --burst-s 0 --quiet-s 0 --component-s 0 --pmc none --out "$OUT/trainpmfw.json" ;;
    train2) run train2 600 python -u bench.py --load train --steps 10 --warmup 2 --rounds 32 --hz-list 100 \
              --capacity-hz "" --burst-s 0 --quiet-s 0 --component-s 0 --pmc-lean 2 --out "$OUT/train2.json" ;;
    tdef|tdef2|tpmfw|tagent|tl3agent|tnop|t1k|tbatch*|tpub*|tnobatch|tnobatch2|t16k)
        # training-step side runs, 36 rounds = every block order 6 times:
        #   tdef (defaults) tpmfw (no READs) tagent (release fence at agent scope)
        #   tl3agent (lean 3 + agent release) tnop (every READ packet a NOP: the bare
        #   packet's cost; values stale) t1k (1 kHz tier)
        T=(python -u bench.py --load train --steps 10 --warmup 2 --rounds 36 --hz-list 100 --capacity-hz ""
           --burst-s 0 --quiet-s 0 --component-s 0 --util-s 0 --out "$OUT/$s.json")
        case $s in
          tdef|tdef2) run $s 600 "${T[@]}" ;;
          tpmfw) run $s 600 "${T[@]}" --pmc none ;;
          tagent) KGS_AQL_FENCE=none,agent run $s 600 "${T[@]}" ;;
          tl3agent) KGS_AQL_FENCE=none,agent KGS_AQL_LEAN=3 run $s 600 "${T[@]}" ;;
          tnop) KGS_AQL_LEAN=5 run $s 600 "${T[@]}" ;;
          t1k) run $s 600 "${T[@]}" --hz 1000 ;;
          tbatch*) run $s 600 "${T[@]}" --pmc-batch "${s#tbatch}" ;;      # tbatch8: --pmc-batch 8
          tpub*) run $s 600 "${T[@]}" --pmc-publish-us "${s#tpub}" ;;     # tpub0: count-only batches
          tnobatch|tnobatch2) run $s 600 "${T[@]}" --pmc-batch 1 ;;
          t16k) run $s 600 "${T[@]}" --hz 16000 --pmc-batch 16 ;;
        esac ;;
    bpub*) run $s 600 python -u bench.py --steps 20 --warmup 5 --pmc-publish-us "${s#bpub}" --out "$OUT/$s.json" ;;
    b16k) run $s 600 python -u bench.py --steps 20 --warmup 5 --hz 16000 --pmc-batch 16 --out "$OUT/$s.json" ;;
    b16knd) KGS_TICK_DITHER=0 run $s 600 python -u bench.py --steps 20 --warmup 5 --hz 16000 --pmc-batch 16 \
              --out "$OUT/$s.json" ;;  # the 16 kHz tier on a fixed tick grid
    bnd) KGS_TICK_DITHER=0 run $s 600 python -u bench.py --steps 20 --warmup 5 --out "$OUT/$s.json" ;;
    bnobatch|bnobatch2) run $s 600 python -u bench.py --steps 20 --warmup 5 --pmc-batch 1 --out "$OUT/$s.json" ;;
    bbatch*) run $s 600 python -u bench.py --steps 20 --warmup 5 --pmc-batch "${s#bbatch}" --out "$OUT/$s.json" ;;
    soak) run soak 420 python -u tools/soak.py --seconds 240 --out "$OUT/soak.json" ;;
    rss) run rss 180 python -u tools/rss_probe.py --out "$OUT/rss_probe.json" ;;
    hsarss) run hsarss 300 python -u tools/hsa_rss_probe.py --out "$OUT/hsa_rss.json" ;;
    soakpark) run soakpark 360 python -u tools/soak.py --seconds 180 --idle-s 4 --quiet-release-s 2 \
                --out "$OUT/soakpark.json" ;;
    soak90) run soak90 240 python -u tools/soak.py --seconds 90 --out "$OUT/soak90.json" ;;
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider ;;
    # round 4
    smprobe) run sm_util_probe 300 python -u tools/sm_util_probe.py --out "$OUT/sm_util_probe.json" ;;
    cpprobe) run cp_busy_probe 240 python -u tools/cp_busy_probe.py --out "$OUT/cp_busy_probe.json" ;;
    cpdump) run cp_dump 300 python -u tools/cp_busy_probe.py --rates 8000,1000 --pipelined 1 --secs 2 \
              --out "$OUT/cp_busy_pipelined.json" --dump "$OUT/cp_dump.json" --dump-rates 8000,1000 ;;
    graphutil) run graph_util 300 python -u tools/graph_cost_probe.py --variants full_rate,util_set,lite,default \
                 --out "$OUT/graph_util.json" ;;
    cpdumplite) run cp_dump_lite 300 python -u tools/cp_busy_probe.py --rates 8000,1000 --pipelined 1 --batch 8 \
                  --lite 1 --exporter-set 1 --secs 2 --out "$OUT/cp_busy_lite.json" --dump "$OUT/cp_dump_lite.json" \
                  --dump-rates 8000,1000 ;;
    graphdef) run graph_def 300 python -u tools/graph_cost_probe.py --variants default,nolite,lite \
                --out "$OUT/graph_def.json" ;;
    graphcost) run graph_cost 400 python -u tools/graph_cost_probe.py --out "$OUT/graph_cost.json" ;;
    testsnw) run pytest_gpu 700 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread \
               -p no:cacheprovider -k "not wedged_counter_queue" ;;
    testsdb) run pytest_dbound 400 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread \
               -p no:cacheprovider -k "dispatch_bound or read_immune" ;;
    testslite) run pytest_lite 300 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread \
                 -p no:cacheprovider -k "lite_reads or dispatch_bound or two_tenants" ;;
    # round 5
    testsutil) run pytest_util 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
                 -p no:cacheprovider -k "shipped_daemonset or read_immune or lite_reads or mfma_kernel" ;;
    cpdumpall) run cp_dump_all 420 python -u tools/cp_busy_probe.py --rates 8000,1000,100,10 --pipelined 1 --batch 8 \
                 --lite 1 --exporter-set 1 --secs 4 --out "$OUT/cp_busy_all.json" --dump "$OUT/cp_dump_all.json" \
                 --dump-rates 8000,1000,100,10 ;;
    umcprobe) KGS_AQL_PROBE_OUT="$OUT/aql_probe_mem.json" run aql_probe_mem 300 python -u tools/aql_probe.py \
                umc_a,umc_b,mmea,gcea ;;
    gceaprobe) KGS_AQL_PROBE_OUT="$OUT/aql_probe_gcea.json" run aql_probe_gcea 400 python -u tools/aql_probe.py \
                gcea0,gcea1,gcea2,gcea3,gcea4,gcea5,gcea6,gcea7 ;;
    utilonly*) run $s 300 python -u bench.py --steps 5 --warmup 2 --rounds 2 --burst-s 0 --capacity-hz "" \
                 --quiet-s 0 --component-s 0 --util-s 3 --out "$OUT/$s.json" ;;  # phase U, 8 kHz / 1 kHz / 10 Hz
    phase) run phase_8k 200 python -u tools/phase_probe.py --out "$OUT/phase_8k.json"
           run phase_8k_1ms 200 python -u tools/phase_probe.py --burst-ms 1 --period-ms 5 --out "$OUT/phase_8k_1ms.json" ;;
    phaselow) run phase_1k 200 python -u tools/phase_probe.py --hz 1000 --out "$OUT/phase_1k.json"
              run phase_100 300 python -u tools/phase_probe.py --hz 100 --burst-ms 1 --period-ms 5 --window-s 2 \
                --windows 10 --out "$OUT/phase_100.json" ;;
    lowrate) run lowrate_10 90 python -u tools/lowrate_probe.py --hz 10 --out "$OUT/lr_10.json"
             run lowrate_10_sat 60 python -u tools/lowrate_probe.py --hz 10 --burst-ms 3000 --period-ms 3000 \
               --load-s 3 --out "$OUT/lr_10_sat.json"
             run lowrate_100 60 python -u tools/lowrate_probe.py --hz 100 --out "$OUT/lr_100.json" ;;
    # round 6: the driver's own invocation (one process, -x), and the same without -x
    testsx) run pytest_gpu_x 900 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread \
              -p no:cacheprovider -rA ;;
    testsall) run pytest_gpu_all 900 python -u -m pytest tests -q -m gpu -v --timeout 150 --timeout-method thread \
                -p no:cacheprovider -rA ;;
    cpdumpirr) run cp_dump_irregular 420 python -u tools/cp_busy_probe.py --rates 8000,1000,100,10 --pipelined 1 \
                 --batch 8 --lite 1 --exporter-set 1 --secs 4 --irregular 1 --only-irregular 1 \
                 --out "$OUT/cp_busy_irregular.json" --dump "$OUT/cp_dump_irregular.json" --dump-rates 8000,1000,100,10 ;;
    testsirr) run pytest_irregular 300 python -u -m pytest tests -m gpu -v --timeout 250 --timeout-method thread \
                -p no:cacheprovider -rA -k "irregular" ;;
    poweronly) run poweronly 600 python -u bench.py --steps 5 --warmup 2 --rounds 0 --burst-s 0 --capacity-hz "" \
                 --quiet-s 0 --component-s 0 --util-s 0 --idle-power-s 60 --idle-power-rounds 6 --out "$OUT/poweronly.json" ;;
    testspark) run pytest_park 200 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread \
                 -p no:cacheprovider -rA -k "quiet_release" ;;
    powerabs) run powerabs 720 python -u bench.py --steps 5 --warmup 2 --rounds 0 --burst-s 0 --capacity-hz "" \
                --quiet-s 0 --component-s 0 --util-s 0 --idle-power-s 64 --idle-power-rounds 8 --idle-power-absent 1 \
                --out "$OUT/powerabs.json" ;;
    tierprobe) run idle_tier 600 python -u tools/idle_tier_probe.py --out "$OUT/idle_tier_probe.json" ;;
    tierprobe60) run idle_tier60 840 python -u tools/idle_tier_probe.py --secs 60 --out "$OUT/idle_tier_probe60.json" ;;
    useeds) for s in 1 2 3 4 5 6 7 8; do
              run useed_$s 240 python -u bench.py --steps 3 --warmup 1 --rounds 0 --burst-s 0 --capacity-hz "" \
                --quiet-s 0 --component-s 0 --idle-power-s 0 --util-hz 10 --util-seed $s --out "$OUT/useed_$s.json" || break
            done ;;
    kfdprobe) run kfd_proc 120 python -u tools/kfd_proc_probe.py --out "$OUT/kfd_proc.json" ;;
    wedge) run pytest_wedge 150 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
             -p no:cacheprovider -k wedged_counter_queue ;;
    smoke) run smoke 180 python -u __graft_entry__.py smoke ;;
    bench) run bench 900 python -u bench.py --steps 20 --warmup 5 --out "$OUT/bench.json" ;;
    bench2) run bench_b 600 python -u bench.py --steps 20 --warmup 5 --out "$OUT/bench_b.json" ;;
    rocprof) run rocprof 1000 bash tools/gpu_rocprof.sh "$OUT/rocprof" ;;
  esac
done
echo "== done $(date +%T)"
