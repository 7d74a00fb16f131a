"""Print the tail of a rocprofv3 kernel trace as a timeline (us from a reference
point): start, end, duration, queue, kernel (short name), grid."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(name):
    for key, tag in (("copy_pieces", "COPY"), ("gf_apply_bytes", "bytes"), ("hash_reduce", "hred"),
                     ("gf_apply_lens", "lens"), ("gf_apply", "code"), ("fillBuffer", "fill"), ("copyBuffer", "blit"),
                     ("streamOps", "sops")):
        if key in name:
            return tag
    return name[:20]


rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} - {(e - t0) / 1e3:9.1f} dur {(e - s) / 1e3:8.1f} q{r['Queue_Id']:>2} "
          f"{short(r['Kernel_Name']):6s} grid {r['Grid_Size_X']}")
