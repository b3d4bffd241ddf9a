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
    if commit is None:
        # tools/gpu.sh sq / sqlds write the measured commit next to the pass
        import os
        d = os.path.dirname(os.path.abspath(path))
        for _ in range(3):
            f = os.path.join(d, "commit.txt")
            if os.path.exists(f):
                commit = open(f).read().strip() or None
                break
            d = os.path.dirname(d)
    rows = collections.defaultdict(list)
    name = None
    for r in csv.DictReader(open(path)):
        if match in r["Kernel_Name"]:
            name = r["Kernel_Name"]
            rows[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in rows.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    derived = {}
    if "SQ_WAIT_ANY" in avg:  # pass 1 (SQ1): wave-cycle split, bank conflicts
        derived.update({
            "wait_any_frac": avg.get("SQ_WAIT_ANY", 0.0) / wc,
            "wait_inst_any_frac": avg.get("SQ_WAIT_INST_ANY", 0.0) / wc,
            "active_inst_frac": avg.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
            "wait_inst_lds_frac": avg.get("SQ_WAIT_INST_LDS", 0.0) / wc,
            "lds_bank_conflict_per_lds_active":
                avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / (avg.get("SQ_LDS_IDX_ACTIVE", 0.0) or 1.0),
        })
    waves = avg.get("SQ_WAVES", 0.0)
    if waves:  # pass 2 (SQ2): instructions per wave, LDS address conflicts
        lds = avg.get("SQ_INSTS_LDS", 0.0)
        derived.update({
            "valu_per_wave": avg.get("SQ_INSTS_VALU", 0.0) / waves,
            "salu_per_wave": avg.get("SQ_INSTS_SALU", 0.0) / waves,
            "lds_per_wave": lds / waves,
            "lds_addr_conflict_per_lds_inst": avg.get("SQ_LDS_ADDR_CONFLICT", 0.0) / (lds or 1.0),
            "lds_unaligned_stall_per_lds_inst":
                avg.get("SQ_LDS_UNALIGNED_STALL", 0.0) / (lds or 1.0),
            "busy_cycles": avg.get("SQ_BUSY_CYCLES", 0.0),
            "wave_cycles_per_wave": wc / waves,
        })
    res = {"kernel": name, "dispatches": max((len(v) for v in rows.values()), default=0),
           "avg_per_dispatch": avg, "derived": derived, "commit": commit, "source": path}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(derived))


if __name__ == "__main__":
    main()
