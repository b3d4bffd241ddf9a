"""SQ counter pass summary (tools/gpu.sh sq / sqlds recipes): per
kernel the average per dispatch of each counter plus the derived wave-cycle
split. Usage: python3 tools/sq_summary.py <counter_collection.csv> <match>
<out.json> [commit]"""
import collections
import csv
import json
import sys


def main():
    path, match, out = sys.argv[1:4]
    commit = sys.argv[4] if len(sys.argv) > 4 else None
    rows = collections.defaultdict(list)
    name = None
    for r in csv.DictReader(open(path)):
        if match in r["Kernel_Name"]:
            name = r["Kernel_Name"]
            rows[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in rows.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    derived = {
        "wait_any_frac": avg.get("SQ_WAIT_ANY", 0.0) / wc,
        "wait_inst_any_frac": avg.get("SQ_WAIT_INST_ANY", 0.0) / wc,
        "active_inst_frac": avg.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
        "lds_bank_conflict_per_lds_active":
            avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / (avg.get("SQ_LDS_IDX_ACTIVE", 0.0) or 1.0),
    }
    res = {"kernel": name, "dispatches": max((len(v) for v in rows.values()), default=0),
           "avg_per_dispatch": avg, "derived": derived, "commit": commit, "source": path}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(derived))


if __name__ == "__main__":
    main()
