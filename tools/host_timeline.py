"""Timeline of the last host round trip in a rocprofv3 --sys-trace of tools/host_trace.py:
HIP API calls on the host thread, copies and kernels on the device, relative to the start of
the last nic_encode_host call's first copy.  usage: python tools/host_timeline.py <trace dir>"""
import csv
import glob
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    d = sys.argv[1]
    k = rows(f"{d}/**/*kernel_trace.csv")
    m = rows(f"{d}/**/*memory_copy_trace.csv")
    api = rows(f"{d}/**/*hip_api_trace.csv")
    ev = [("K", r["Kernel_Name"][:48], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in k]
    ev += [("C", r.get("Direction", r.get("Operation", "copy")) + " " + r.get("Size", ""), int(r["Start_Timestamp"]),
            int(r["End_Timestamp"])) for r in m]
    ev += [("A", r["Function"][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api
           if r["Function"] in ("hipMemcpyAsync", "hipEventSynchronize", "hipStreamSynchronize", "hipLaunchKernel",
                                "hipStreamWaitEvent", "hipEventRecord", "hipHostMalloc", "hipMemcpy")]
    ev.sort(key=lambda e: e[2])
    copies = [e for e in ev if e[0] == "C"]
    if not copies:
        print("no copies traced")
        return
    # the last round trip: its first copy is the 4th-from-last H2D block start (4 chunks enc + 4 dec)
    h2d = [e for e in copies if "HOST_TO_DEVICE" in e[1].upper() or "H2D" in e[1].upper()]
    t0 = h2d[-8][2] if len(h2d) >= 8 else copies[0][2]
    t_end = max(e[3] for e in ev)
    for kind, name, s, e in ev:
        if s >= t0 - 200000:
            print(f"{kind} {(s - t0) / 1000:9.1f} {(e - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  {name}")
    print("span us", (t_end - t0) / 1000)


if __name__ == "__main__":
    main()
