# One gpurun session, by stages (run from the repo root through gpurun):
#   STAGES="tests bench prof2p30 binned pmc" bash tools/gpu_run.sh
# Every GPU step has its own time limit; the first failing step ends the session (its log stays
# under gpurun_out/$TAG). Stages:
#   tests     python -m pytest tests -m gpu, then smoke()
#   bench     the driver's default line (cfg2 with the CPU baseline) and the other bench lines
#   prof2p30  rocprofv3 kernel stats of the dense push at 2^28 and at 2^30 (north-star size)
#   binned    rocprofv3 kernel stats of the binned patterns (zipf, matrix, exchange)
#   newtests  this round's new GPU tests, then the config-shape tests (cfg4 Long/Double, cfg5 full shape)
#   pmccal    PMC calibration per access shape (tools/microbench_pmc.hip, tools/pmc_calibrate.py)
#   bintests  the GPU tests of the binned path, the full-size cases, cfg4 and the exchange
#   ab        bench zipf / matrix / exchange with a previous library (AB_LIB) and the current one
#   abn       the same over several libraries (LIBS="tag=path[,VAR=VALUE...] ..."; tools/variant.py builds variants)
#   dettests  the deterministic / message-order / full-size GPU tests
#   det       tools/det_probe.py (cfg3 deterministic push), timed and under rocprofv3 kernel stats
#   micro     tools/microbench_stream mode 6: the dense sweep at 2^26..2^30, chunked and shifted
#   pmc       FETCH_SIZE / WRITE_SIZE passes (separate runs) of the dense, zipf and matrix lines
#   latency   tools/host_latency.py (per-call cost of the host-pointer entry points)
#   ring      tools/ring_probe.py: pipelined message-sized wire pushes, timed and with kernel stats
#   loopback  tools/loopback/build/glint_loopback, HBM shards vs the oracle's CPU loop (cfg1, cfg4 shapes)
#   lbspin    cfg4b thread-per-connection pulls with GLINT_LOCK_SPIN 0 / 200 / 2000 (a round-5 build knob,
#             removed after this A/B), cfg1 actor rows, CPU loop beside
set -o pipefail
TAG=${TAG:-r06}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
[ -n "$GLINT_GPU_LIB" ] && export GLINT_GPU_LIB=$(realpath "$GLINT_GPU_LIB")  # (kstats / pmc run from /tmp)
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> <command...>: output to $OUT/<name>.log
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] $name" >&2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -30 $OUT/$name.log >&2; exit $rc; fi
}
kstats() {  # kstats <name> <seconds> <bench args...>: kernel stats CSV of one bench command
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] kstats $name" >&2
  (cd /tmp && timeout -k 10 $secs rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run \
     -- python3 $R/bench.py --no-cpu-baseline --no-north-star "$@" > $OUT/prof_$name.log 2>&1) || { tail -30 $OUT/prof_$name.log >&2; exit 1; }
  find /tmp/prof_$name -name "*kernel_stats.csv" -exec cp {} $OUT/kstats_$name.csv \;
}
pmc() {  # pmc <name> <bench args...>: FETCH_SIZE and WRITE_SIZE in two separate passes
  local name=$1
  shift
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "[$(date +%T)] pmc $name $c" >&2
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d /tmp/pmc_${name}_$c -o run \
       -- python3 $R/bench.py --no-cpu-baseline --no-north-star --no-check --steps 5 --warmup 2 "$@" > $OUT/pmc_${name}_$c.log 2>&1) \
       || { tail -30 $OUT/pmc_${name}_$c.log >&2; exit 1; }
    find /tmp/pmc_${name}_$c -name "*counter_collection.csv" -exec cp {} $OUT/pmc_${name}_$c.csv \;
  done
}
for s in ${STAGES:-tests bench}; do
  case $s in
    tests)
      step pytest_gpu 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
      ;;
    bench)
      step bench_default 400 python3 bench.py
      for pat in zipf matrix exchange pull rowpull; do
        step bench_$pat 300 python3 bench.py --no-cpu-baseline --pattern $pat
      done
      step bench_exchange_mps8 300 python3 bench.py --no-cpu-baseline --pattern exchange --parts-per-gpu 8
      ;;
    prof2p30)
      kstats dense_2p28 300 --log2-keys 28
      kstats dense_2p30 400 --log2-keys 30 --steps 10
      ;;
    binned)
      for pat in ${PATTERNS:-zipf matrix exchange}; do kstats $pat 300 --pattern $pat --steps 10 --warmup 2; done
      kstats exchange_mps8 300 --pattern exchange --parts-per-gpu 8 --steps 10 --warmup 2
      ;;
    pmc)
      for w in ${PMC:-dense_2p28 dense_2p30 zipf_2p28 matrix_2p17x512}; do
        case $w in
          dense_2p28) pmc $w --log2-keys 28 ;;
          dense_2p30) pmc $w --log2-keys 30 ;;
          zipf_2p28) pmc $w --pattern zipf ;;
          matrix_2p17x512) pmc $w --pattern matrix ;;
          exchange_2p28) pmc $w --pattern exchange ;;
          exchange_2p28_mps8) pmc $w --pattern exchange --parts-per-gpu 8 ;;
        esac
      done
      ;;
    newtests)  # this round's new GPU tests first (fast feedback), then the config-shape tests
      step pytest_new 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -k "hot_chain or odd_record or scatter_rows or copy_segments or send_matrix or dist_exchange or cfg5_slice or gated"
      step pytest_configs 1100 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 600 --timeout-method thread
      ;;
    pmccal)  # FETCH_SIZE / WRITE_SIZE per access shape against known byte counts (tools/microbench_pmc.hip)
      step pmccal_known 120 tools/build/microbench_pmc
      for c in FETCH_SIZE WRITE_SIZE; do
        echo "[$(date +%T)] pmccal $c" >&2
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d /tmp/pmccal_$c -o run \
           -- $R/tools/build/microbench_pmc > $OUT/pmccal_$c.log 2>&1) || { tail -30 $OUT/pmccal_$c.log >&2; exit 1; }
        find /tmp/pmccal_$c -name "*counter_collection.csv" -exec cp {} $OUT/pmccal_$c.csv \;
      done
      python3 tools/pmc_calibrate.py $OUT/pmccal_known.log $OUT/pmccal_FETCH_SIZE.csv $OUT/pmccal_WRITE_SIZE.csv \
        $OUT/pmc_calibration.json >&2
      ;;
    tailab)  # the unordered tail: atomic scatter vs binned by density, one stream and 8 (tools/tail_ab.py)
      step tail_ab 600 python3 tools/tail_ab.py --reps ${REPS:-10}
      grep '^{' $OUT/tail_ab.log > $OUT/tail_ab.jsonl || true
      ;;
    quickbench)  # the binned lines only, no CPU baseline
      for pat in ${PATTERNS:-matrix zipf exchange}; do
        step qb_$pat 300 python3 bench.py --no-cpu-baseline --no-north-star --pattern $pat
      done
      ;;
    phases)  # phase clocks of the binned kernels (tools/bin_phases.py, a -DGLINT_BIN_PROF build)
      step bin_phases 300 python3 tools/bin_phases.py
      ;;
    lbcpu)  # the cfg4 loopback rows with the process / server-call CPU time (--cpu-stats), both backends
      LB=tools/loopback/build/glint_loopback
      i=0
      for args in "--clients 64 --servers 8 --keys 33554432" \
                  "--clients 64 --servers 8 --keys 33554432 --pattern uniform --records 524288 --dtype long"; do
        for r in $(seq ${ROUNDS:-2}); do
          for lv in ${LBLIBS:-cur=glint_amd/lib/libglint_gpu.so}; do  # tag=path
            step lbc_gpu_${lv%%=*}_${i}_$r 200 $LB --backend gpu --lib ${lv#*=} $args --cpu-stats
          done
          [ -z "$NO_ORACLE" ] && step lbc_oracle_${i}_$r 200 $LB --backend oracle --lib oracle/build/libglint_oracle.so $args --cpu-stats
        done
        i=$((i + 1))
      done
      cat $OUT/lbc_*.log | grep '^{' > $OUT/loopback_cpu.jsonl || true
      ;;
    lbactor)  # the cfg1 / cfg4 loopback rows with --server actor (one thread per server, as the Akka actor), both backends
      LB=tools/loopback/build/glint_loopback
      i=0
      for args in "" "--clients 64 --servers 8 --keys 33554432" \
                  "--clients 64 --servers 8 --keys 33554432 --pattern uniform --records 524288 --dtype long"; do
        for r in $(seq ${ROUNDS:-2}); do
          for ans in ${ANSWERS:-direct}; do  # direct: answers written by the GPU into pinned arenas; copy: malloc'd
            step lba_gpu_${ans}_${i}_$r 200 $LB --backend gpu --lib glint_amd/lib/libglint_gpu.so $args --server actor --answers $ans --cpu-stats
          done
          step lba_oracle_${i}_$r 200 $LB --backend oracle --lib oracle/build/libglint_oracle.so $args --server actor --cpu-stats
        done
        i=$((i + 1))
      done
      cat $OUT/lba_*.log | grep '^{' > $OUT/loopback_actor.jsonl || true
      ;;
    bintests)
      step pytest_binned 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread \
        -k "binned or fullsize or adaptive or cfg4 or exchange"
      ;;
    ab)  # the binned patterns: the previous build's library (GLINT_GPU_LIB=$AB_LIB) and this one, back to back
      for pat in ${PATTERNS:-zipf matrix exchange}; do
        step ab_old_$pat 300 env GLINT_GPU_LIB=$AB_LIB python3 bench.py --no-cpu-baseline --pattern $pat
        step ab_new_$pat 300 python3 bench.py --no-cpu-baseline --pattern $pat
      done
      ;;
    abn)  # LIBS="tag=path ...": each binned pattern on each library, ROUNDS rounds interleaved (one box)
      for r in $(seq ${ROUNDS:-2}); do
        for pat in ${PATTERNS:-zipf matrix exchange}; do
          for lv in $LIBS; do  # tag=path[,VAR=VALUE...]
            spec=${lv#*=}
            extra=""
            case $spec in *,*) extra=$(echo ${spec#*,} | tr ',' ' ') ;; esac
            step ab_${lv%%=*}_${pat}_$r 300 env GLINT_GPU_LIB=${spec%%,*} $extra python3 bench.py --no-cpu-baseline --no-north-star --pattern $pat
          done
        done
      done
      ;;
    dettests)
      step pytest_det 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread \
        -k "determin or order or fullsize or det"
      ;;
    det)  # the deterministic cfg3 push (sort + in-order fold), timed and with kernel stats
      step det_probe 300 python3 tools/det_probe.py
      echo "[$(date +%T)] kstats det" >&2
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_det -o run \
         -- python3 $R/tools/det_probe.py > $OUT/prof_det.log 2>&1) || { tail -30 $OUT/prof_det.log >&2; exit 1; }
      find /tmp/prof_det -name "*kernel_stats.csv" -exec cp {} $OUT/kstats_det.csv \;
      ;;
    micro)
      step micro_stream_2p30 300 tools/microbench_stream 30 9 6
      ;;
    latency)  # per-call cost of the host-pointer entry points, and the box's launch / mapped-wait floor
      step host_latency 300 python3 tools/host_latency.py --reps 300
      ;;
    ring)  # pipelined message-sized wire pushes (4000 x 1000 random keys), timed and under kernel stats
      step ring_probe 300 python3 tools/ring_probe.py 1000 4000
      echo "[$(date +%T)] kstats ring" >&2
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_ring -o run \
         -- python3 $R/tools/ring_probe.py 1000 4000 > $OUT/prof_ring.log 2>&1) || { tail -30 $OUT/prof_ring.log >&2; exit 1; }
      find /tmp/prof_ring -name "*kernel_stats.csv" -exec cp {} $OUT/kstats_ring.csv \;
      ;;
    loopback)  # cfg1 / window 1 / 79 999-record messages / cfg4a / cfg4b over loopback TCP, both backends;
               # the cfg4 shapes also with the client bucketing offloaded to the device route
      LB=tools/loopback/build/glint_loopback
      G="--backend gpu --lib glint_amd/lib/libglint_gpu.so"
      O="--backend oracle --lib oracle/build/libglint_oracle.so"
      i=0
      for args in "" "--window 1" "--keys 16777216 --msg 79999" "--clients 64 --servers 8 --keys 33554432" \
                  "--clients 64 --servers 8 --keys 33554432 --pattern uniform --records 524288 --dtype long"; do
        for r in 1 2; do  # the GPU server twice (one wait per drained burst; LB_ASYNC=1: also with reply threads)
          step lb_gpu_${i}_$r 200 $LB $G $args
          [ -n "$LB_ASYNC" ] && step lb_gpuasync_${i}_$r 200 $LB $G $args --replies async
        done
        step lb_oracle_$i 200 $LB $O $args
        case "$args" in *--clients*) step lb_gpudev_$i 200 $LB $G $args --bucket device ;; esac
        i=$((i + 1))
      done
      cat $OUT/lb_gpu_*.log | grep '^{' > $OUT/loopback_gpu.jsonl || true
      cat $OUT/lb_gpuasync_*.log 2>/dev/null | grep '^{' > $OUT/loopback_gpu_async.jsonl || true
      cat $OUT/lb_gpudev_*.log | grep '^{' > $OUT/loopback_gpu_bucket_device.jsonl || true
      cat $OUT/lb_oracle_*.log | grep '^{' > $OUT/loopback_oracle.jsonl || true
      ;;
    *)
      echo "unknown stage $s" >&2
      exit 2
      ;;
  esac
done
echo "session done" >&2
