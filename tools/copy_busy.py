"""Copy-kernel activity in a rocprofv3 kernel trace of the host path (round 6): over the last 60 % of
the run, the share of time any copy_pieces kernel runs, the share with two or more at once, the gaps
between them and the copy durations.   python tools/copy_busy.py <run_kernel_trace.csv>"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
cp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], int(r["Grid_Size_X"])) for r in rows if "copy_pieces" in r["Kernel_Name"]]
code = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows if "gf_apply" in r["Kernel_Name"]]
other = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:30]) for r in rows if "copy_pieces" not in r["Kernel_Name"] and "gf_apply" not in r["Kernel_Name"]]
# window: last 60% of copy activity
t0 = cp[len(cp)*2//5][0]; t1 = cp[-1][1]
iv = sorted((max(s,t0), min(e,t1)) for s,e,_,_ in cp if e > t0)
busy = 0; cur_s, cur_e = iv[0]; gaps = []
for s, e in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s; gaps.append(s - cur_e); cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
# concurrency: time with >=2 copy kernels
ev = sorted([(s,1) for s,e in iv] + [(e,-1) for s,e in iv])
c = 0; last = ev[0][0]; t2 = 0
for t, d in ev:
    if c >= 2: t2 += t - last
    c += d; last = t
n = len([1 for s,e,_,_ in cp if s >= t0])
print(f"window {(t1-t0)/1e6:.1f} ms, copy launches {n}, busy {busy/(t1-t0)*100:.1f} %, >=2 copies {t2/(t1-t0)*100:.1f} %, gaps {len(gaps)} mean {sum(gaps)/max(1,len(gaps))/1e3:.1f} us max {max(gaps or [0])/1e3:.1f} us")
durs = sorted((e-s)/1e3 for s,e,_,_ in cp if s >= t0)
print("copy durations us: p10 %.0f p50 %.0f p90 %.0f" % (durs[len(durs)//10], durs[len(durs)//2], durs[len(durs)*9//10]))
print("other kernels in window:", len([1 for s,e,n in other if s >= t0]), set(n for s,e,n in other if s>=t0))
