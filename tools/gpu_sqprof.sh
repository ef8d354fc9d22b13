# SQ counters per binned-push kernel (cfg3 Zipf and cfg5 matrix): where the waves wait
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/sq
mkdir -p $OUT
R=$(pwd)
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU"
timeout -k 10 200 python3 bench.py --pattern exchange --no-cpu-baseline > $OUT/bench_exchange.json 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/xtrace -o run -- python3 $R/bench.py --no-cpu-baseline --pattern exchange --steps 10 --no-check > $R/$OUT/exchange_traced.txt 2>&1 || exit 1
for pat in zipf matrix; do
  timeout -s KILL 120 rocprofv3 --pmc $A --output-format csv -d $R/$OUT/${pat}_a -o run -- python3 $R/bench.py --no-cpu-baseline --pattern $pat --steps 3 --warmup 1 --no-check > $R/$OUT/${pat}_a.txt 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $B --output-format csv -d $R/$OUT/${pat}_b -o run -- python3 $R/bench.py --no-cpu-baseline --pattern $pat --steps 3 --warmup 1 --no-check > $R/$OUT/${pat}_b.txt 2>&1 || exit 1
done
