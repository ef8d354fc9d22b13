# pipelined message-sized wire pushes: wall time per message, then the kernel stats of the same run
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python3 $R/tools/ring_probe.py 1000 4000 > $R/gpurun_out/ring_probe.txt 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rp -o run -- python3 $R/tools/ring_probe.py 1000 4000 > $R/gpurun_out/ring_probe_traced.txt 2>&1
find /tmp/rp -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/kstats_ring.csv \;
rm -rf /tmp/rp
