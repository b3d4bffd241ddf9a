#!/usr/bin/env python3
"""Which hardware queue each HIP stream's dispatches landed on, from a
rocprofv3 kernel trace (tools/c5trace.sh): (queue, stream) pairs in order of
first dispatch with the first kernel's name, and the ogs_ kernels' count per
(queue, stream).  python tools/queue_map.py <kernel_trace.csv> ..."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    first = collections.OrderedDict()
    ogs = collections.Counter()
    for r in rows:
        k = (int(r["Queue_Id"]), int(r["Stream_Id"]))
        first.setdefault(k, r["Kernel_Name"][:48])
        if "ogs::" in r["Kernel_Name"]:
            ogs[k] += 1
    print(path)
    for (q, s), name in first.items():
        print(f"  queue {q} stream {s}: first {name!r}, ogs kernels {ogs[(q, s)]}")
