"""Where one C4 frame's time goes, from a rocprofv3 kernel trace of
`bench.py --config c4` (tools/ab/gpu_c4_trace.sh): frames are delimited by
the camera-rays kernel; per frame the wall time, the device busy time (union
of kernel intervals), the idle gaps, and busy time per kernel name."""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "rays_kernel" in r["Kernel_Name"]]
for k in range(1, len(starts) - 1):
    seg = rows[starts[k]:starts[k + 1]]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg)
    busy, (cs, ce) = 0, iv[0]
    gaps = []
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append(s - ce)
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    per = collections.Counter()
    cnt = collections.Counter()
    for r in seg:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        per[name] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        cnt[name] += 1
    print(f"frame {k}: wall {(t1 - t0) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, idle "
          f"{sum(gaps) / 1e6:.2f} ms in {len(gaps)} gaps (>20 us: "
          f"{sum(g for g in gaps if g > 20000) / 1e6:.2f} ms), {len(seg)} kernels")
    for name, t in per.most_common(12):
        print(f"   {t / 1e6:8.2f} ms  {cnt[name]:4d}x  {name}")
