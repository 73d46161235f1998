"""Summarize a tools/profile_pmc.sh output directory (derived metrics per the MI355X guide)."""
import csv, glob, json, sys
d = sys.argv[1]
vals, meta = {}, {}
for f in sorted(glob.glob(f"{d}/g*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
        meta = {k: r[k] for k in ("Kernel_Name", "VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Scratch_Size")}
g = lambda k: vals.get(k, float("nan"))
xcd_cycles = g("GRBM_GUI_ACTIVE") / 8
der = {
    "valu_lane_utilization": g("SQ_THREAD_CYCLES_VALU") / (g("SQ_ACTIVE_INST_VALU") * 64),
    "avg_waves_per_simd": g("SQ_WAVE_CYCLES") * 4 / 1024 / xcd_cycles,
    "wait_mem_frac": g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"),
    "wait_issue_frac": g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"),
    "active_frac": g("SQ_ACTIVE_INST_ANY") / g("SQ_WAVE_CYCLES"),
    "valu_insts": g("SQ_INSTS_VALU"), "vmem_rd_insts": g("SQ_INSTS_VMEM_RD"), "lds_insts": g("SQ_INSTS_LDS"),
    "salu_insts": g("SQ_INSTS_SALU"), "branch_insts": g("SQ_INSTS_BRANCH"),
    "ta_busy_frac_per_cu": g("TA_TA_BUSY_sum") / 256 / xcd_cycles,
    "l1_miss_frac": g("TCP_TCC_READ_REQ_sum") / max(1, g("TCP_TOTAL_CACHE_ACCESSES_sum")),
    "lds_bank_conflict_cycles": g("SQ_LDS_BANK_CONFLICT"),
    "hbm_read_bytes(FETCH_SIZE*1024*2, gfx950 1/2 correction)": g("FETCH_SIZE") * 1024 * 2,
    "hbm_write_bytes(WRITE_SIZE*1024)": g("WRITE_SIZE") * 1024,
    "kernel_clock_ghz_est": None,
    "vmem_latency_cycles": g("SQ_INST_LEVEL_VMEM") / g("SQ_INSTS_VMEM"),
    "lds_latency_cycles": g("SQ_INST_LEVEL_LDS") / g("SQ_INSTS_LDS"),
    "icache_miss_per_ifetch": g("SQC_ICACHE_MISSES") / g("SQ_IFETCH"),
    "ta_addr_fifo_full_frac": g("SQ_VMEM_TA_ADDR_FIFO_FULL") / 256 / xcd_cycles,
    "ta_cmd_fifo_full_frac": g("SQ_VMEM_TA_CMD_FIFO_FULL") / 256 / xcd_cycles,
    "valu_trans_frac": g("SQ_INSTS_VALU_TRANS_F32") / g("SQ_INSTS_VALU"),
}
out = {"kernel": meta, "derived": der, "counters": vals}
print(json.dumps(out, indent=1))
