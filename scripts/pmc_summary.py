"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc_r2.sh) per kernel: MFMA busy share, wave wait
share, HBM fetch / write bytes and rates (FETCH_SIZE / WRITE_SIZE are in KB)."""
import collections
import csv
import glob
import sys


def load(d):
    fs = glob.glob(f"{d}/*/*counter_collection.csv")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for row in csv.DictReader(open(fs[0])):
        k = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        dur[k][row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    return agg, {k: sum(v.values()) for k, v in dur.items()}


def main(root="gpurun_out/pmc", names="mftopk,w2v,mf", top="4"):
    print("| run | kernel | time (s, pass 1) | MFMA busy | waves waiting | LDS bank conflict / LDS active | HBM read | HBM write "
          "| read+write rate | of 8 TB/s |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name in names.split(","):
        a1, t1 = load(f"{root}/{name}_1")
        a2, t2 = load(f"{root}/{name}_2")
        a3, t3 = load(f"{root}/{name}_3")
        for k in sorted(a1, key=lambda k: -t1.get(k, 0))[:int(top)]:
            c = a1[k]
            gui = c.get("GRBM_GUI_ACTIVE", 0) / 8  # summed over the 8 XCDs
            busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / gui if gui else 0  # per SIMD
            wait = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else 0
            rd = a2.get(k, {}).get("FETCH_SIZE", 0) * 1024
            wr = a3.get(k, {}).get("WRITE_SIZE", 0) * 1024
            rate = (rd / t2[k] if t2.get(k) else 0) + (wr / t3[k] if t3.get(k) else 0)
            lds = c.get("SQ_LDS_IDX_ACTIVE", 0)
            conf = f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:.1%}" if lds else "no LDS"
            print(f"| {name} | `{k}` | {t1.get(k, 0):.4f} | {busy:.0%} | {wait:.0%} | {conf} | {rd / 1e9:.2f} GB "
                  f"| {wr / 1e9:.2f} GB | {rate / 1e12:.2f} TB/s | {rate / 8e12:.0%} |")


if __name__ == "__main__":
    main(*sys.argv[1:])
