#!/usr/bin/env python3
"""Prints the last N dispatches of a rocprofv3 kernel trace (csv) as a
timeline: start / end offsets (us) from the first of them, duration, queue,
short kernel name (runtime copies / torch kernels left out). Usage: trace_timeline.py <k_kernel_trace.csv> [N]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rows = [r for r in rows if "rocclr" not in r["Kernel_Name"] and
            "elementwise" not in r["Kernel_Name"] and "reduce" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"].split("(")[0][:60]
        print(f"{s / 1e3:9.2f} {e / 1e3:9.2f} {(e - s) / 1e3:8.2f} q{r['Queue_Id']} "
              f"grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} wg={r['Workgroup_Size_X']} "
              f"lds={r['LDS_Block_Size']} {name}")


if __name__ == "__main__":
    main()
