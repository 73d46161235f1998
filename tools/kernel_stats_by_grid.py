"""rocprofv3 kernel-trace summary split by (kernel, grid size): the default bench run launches the same kernel
instantiation for C2 (32400 tiles) and C3 (129600 tiles), which rocprofv3's --stats averages together.
    python tools/kernel_stats_by_grid.py gpurun_out/prof/bench_kernel_trace.csv > profiles/<round>_kernel_stats_by_grid.csv"""
import collections, csv, statistics, sys

groups = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    groups[(r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
w = csv.writer(sys.stdout)
w.writerow(["Name", "Grid_Size_X", "Workgroup_Size_X", "Calls", "AverageMs", "MedianMs", "MinMs", "MaxMs"])
for (name, grid, wg), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([name, grid, wg, len(d), round(statistics.mean(d), 4), round(statistics.median(d), 4),
                round(min(d), 4), round(max(d), 4)])
