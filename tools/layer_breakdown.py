#!/usr/bin/env python3
"""Per-position kernel timing of one U-Net evaluation from a rocprofv3 kernel-trace CSV."""
import collections, csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'tcx' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
seq, cur = [], []
# an evaluation starts at k_cond (per-evaluation conditioning) or, when the sampler hoisted it
# (k_cond_maps once per call), at the first conv
starts = 'k_cond(' if any('k_cond(' in r['Kernel_Name'] for r in rows) else 'k_conv_first'
if starts == 'k_conv_first':  # round 3: statistics pass <1> then record pass <2>; the fp32 form <0>
    starts = next((s for s in ('k_conv_first<1>', 'k_conv_first<0>') if any(s in r['Kernel_Name'] for r in rows)), starts)
for r in rows:
    if starts in r['Kernel_Name']:
        if cur:
            seq.append(cur)
        cur = []
    cur.append(r)
seq.append(cur)
L = collections.Counter(len(s) for s in seq).most_common(1)[0][0]
ev = [s for s in seq if len(s) == L][5:]
tot = 0
for i in range(L):
    d = sum(int(s[i]['End_Timestamp']) - int(s[i]['Start_Timestamp']) for s in ev) / len(ev)
    tot += d
    r0 = ev[0][i]
    nm = r0['Kernel_Name'].split('::')[-1][:60]
    print(f"{i:2d} {nm:60s} grid={r0['Grid_Size_X']:>8s}x{r0['Grid_Size_Y']:<4s} {d / 1e3:9.1f} us")
gaps = sum(int(s[-1]['End_Timestamp']) - int(s[0]['Start_Timestamp']) for s in ev) / len(ev)
print(f"sum of kernels {tot / 1e3:.1f} us; first-start..last-end {gaps / 1e3:.1f} us per eval ({len(ev)} evals)")
