"""Per-kernel durations and idle gaps of one timed step from a rocprofv3
kernel trace (tools/step_gaps.py <run_kernel_trace.csv> [step index])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
       r["Kernel_Name"].replace("void ", "").replace("psamd::(anonymous namespace)::", "")[:34],
       int(r["Grid_Size_X"])) for r in rows]
wi = [i for i, k in enumerate(ks) if k[2].startswith("k_window_init")]
j = int(sys.argv[2]) if len(sys.argv) > 2 else len(wi) // 2
a, b = wi[j], wi[j + 1]
seg = ks[a:b]
print(f"step {j}/{len(wi)}: span {(ks[b][0] - seg[0][0]) / 1e3:.1f} us, "
      f"kernels {sum(e - s for s, e, _, _ in seg) / 1e3:.1f} us")
for i, (s, e, n, g) in enumerate(seg):
    gap = (s - seg[i - 1][1]) / 1e3 if i else 0.0
    print(f"{n:34s} grid={g:8d} dur={(e - s) / 1e3:8.2f} gap={gap:6.2f}")
print(f"{'(next step)':34s} gap={(ks[b][0] - seg[-1][1]) / 1e3:6.2f}")
