"""One step of a bench line from a rocprofv3 trace: every kernel and copy between two consecutive
starts of a marker kernel (default route_hist, one per exchange step), with start / end / duration in
microseconds from the step's start and the hardware queue.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run -- python3 bench.py ...
    python tools/trace_step.py DIR [step index, default -2] [marker kernel substring]
"""
import csv, sys, glob
d = sys.argv[1]
marker = sys.argv[3] if len(sys.argv) > 3 else 'route_hist'
kt = glob.glob(d + '/*kernel_trace.csv')[0]
ev = []
for r in csv.DictReader(open(kt)):
    ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K', r['Kernel_Name'].replace('(anonymous namespace)::','').split('(')[0].replace('void ','')[-50:], r.get('Queue_Id', r.get('Stream_Id', ''))))
mc = glob.glob(d + '/*memory_copy_trace.csv')
if mc:
    for r in csv.DictReader(open(mc[0])):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'C', r.get('Direction', '') + ' ' + r.get('Bytes', r.get('Size', '')), ''))
ev.sort()
starts = [e[0] for e in ev if marker in e[3]]
print(len(starts), marker)
i = int(sys.argv[2]) if len(sys.argv) > 2 else -2
t0, t1 = starts[i], starts[i + 1] if i + 1 < len(starts) else ev[-1][1]
for e in ev:
    if t0 <= e[0] < t1:
        print(f"{(e[0]-t0)/1e3:9.1f} {(e[1]-t0)/1e3:9.1f} {(e[1]-e[0])/1e3:8.1f} {e[2]} {e[4]:>3} {e[3]}")
print('step', (t1 - t0) / 1e3)
