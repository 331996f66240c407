"""Per-step kernel durations and the idle gaps between consecutive kernels from a rocprofv3
--kernel-trace CSV (one encode+decode step, starting at the colour pre-pass).
usage: python tools/trace_gaps.py <kernel_trace.csv> [step index]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else -5
    starts = [i for i, r in enumerate(rows) if "colour_split" in r["Kernel_Name"]]
    i0, i1 = starts[k - 1], starts[k]
    tot_k = tot_gap = 0
    prev_end = None
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = s - prev_end if prev_end is not None else 0
        print(f"{r['Kernel_Name'][:64]:64s} dur {(e - s) / 1000:8.1f} us  gap {gap / 1000:6.1f} us")
        tot_k += e - s
        tot_gap += gap
        prev_end = e
    span = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1000
    print(f"kernels {tot_k / 1000:.1f} us, gaps {tot_gap / 1000:.1f} us, step span {span:.1f} us")


if __name__ == "__main__":
    main()
