"""Summarise tools/pmc_pipe.sh output: per trace-kernel launch averages of every
counter collected, plus the derived busy fractions.

  python tools/pipe_summary.py gpurun_out/pipe_hb
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    agg = collections.defaultdict(list)
    dur = []
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if "trace_kernel" not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: sum(v) / len(v) for k, v in agg.items()}
    for k in sorted(c):
        print(f"{k:40s} {c[k]:16.1f}  ({len(agg[k])} launches)")
    xcd = 8
    cus = 256
    if "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / xcd
        print(f"\nkernel cycles (GRBM_GUI_ACTIVE / 8 XCDs)      {cyc:12.0f}")
        if "TA_BUSY_avr" in c:
            print(f"TA busy fraction                              {c['TA_BUSY_avr'] / cyc:12.3f}")
        if "TA_BUFFER_READ_WAVEFRONTS_sum" in c:
            w = c["TA_BUFFER_READ_WAVEFRONTS_sum"] / cus
            print(f"buffer-load wave instructions per CU          {w:12.0f}   ({c.get('TA_BUSY_avr', 0) / w:.1f} TA-busy cycles each)")
        for k in ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum", "TCP_PENDING_STALL_CYCLES_sum",
                  "TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TD_TD_BUSY_sum", "TD_TC_STALL_sum"):
            if k in c:
                print(f"{k:40s} per CU per cycle {c[k] / cus / cyc:8.3f}")
    if "TCP_UTCL1_REQUEST_sum" in c:
        req = c["TCP_UTCL1_REQUEST_sum"]
        miss = c.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0.0)
        print(f"UTCL1 translation miss rate (MISS / REQUEST)   {miss / max(req, 1.0):12.4f}")
        if "TCP_TCC_READ_REQ_sum" in c:
            print(f"UTCL1 misses per L1->L2 line request          {miss / max(c['TCP_TCC_READ_REQ_sum'], 1.0):12.4f}")
        if "GRBM_UTCL2_BUSY" in c and "GRBM_GUI_ACTIVE" in c:
            print(f"UTCL2 busy fraction (GRBM_UTCL2_BUSY / GUI)   {c['GRBM_UTCL2_BUSY'] / c['GRBM_GUI_ACTIVE']:12.3f}")
        if "GRBM_GUI_ACTIVE" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / xcd
            for k in ("TCP_UTCL1_STALL_MULTI_MISS_sum", "TCP_UTCL1_SERIALIZATION_STALL_sum", "TCP_UTCL1_STALL_LFIFO_NO_RES_sum",
                      "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum", "TCP_PENDING_STALL_CYCLES_sum"):
                if k in c:
                    print(f"{k:40s} per CU per cycle {c[k] / cus / cyc:8.4f}")
    if "SQ_WAVE_CYCLES" in c:
        for k in ("SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_VMEM_TA_CMD_FIFO_FULL",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_VALU"):
            if k in c:
                print(f"{k:40s} / SQ_WAVE_CYCLES {c[k] / c['SQ_WAVE_CYCLES']:8.3f}")
    if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        # a wave64 VALU op occupies a 16-lane SIMD 4 cycles; 4 SIMDs per CU
        print(f"VALU busy (INSTS_VALU x 4 cycles / SIMD cycles)  {c['SQ_INSTS_VALU'] * 4 / (cus * 4) / cyc:.3f}")
    if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
        print(f"VALU lane utilisation (THREAD_CYCLES / 64 / ACTIVE_INST) {c['SQ_THREAD_CYCLES_VALU'] / 64 / c['SQ_ACTIVE_INST_VALU']:.3f}")


if __name__ == "__main__":
    main()
