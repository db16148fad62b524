"""Per-dispatch summary of a rocprofv3 --pmc directory holding the gather roofline's counters
(bench.py GATHER_COUNTERS): duration, TCP tag accesses, L1->L2 read requests, accesses per CU
cycle, TD busy fraction and the clock (GRBM active cycles per XCD / duration).

  python tools/pmc_summary.py <dir with pmc_counter_collection.csv and pmc_kernel_trace.csv>"""
import csv, collections, sys
d = sys.argv[1]
rows = list(csv.DictReader(open(d + "/pmc_counter_collection.csv")))
tr = {r["Dispatch_Id"]: r for r in csv.DictReader(open(d + "/pmc_kernel_trace.csv"))}
per = collections.defaultdict(dict); names = {}
for r in rows:
    per[r["Dispatch_Id"]][r["Counter_Name"]] = per[r["Dispatch_Id"]].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    names[r["Dispatch_Id"]] = r["Kernel_Name"][:40]
for k in sorted(per, key=int):
    t = tr.get(k)
    dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e6 if t else 0
    c = per[k]
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
    acc = c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0); req = c.get("TCP_TCC_READ_REQ_sum", 0)
    td = c.get("TD_TD_BUSY_sum", 0) / 256
    if "fill" in names[k]: continue
    print("%3s %-40s %.4f ms  acc %.4g  req %.4g  acc/CUcyc %.3f  TDbusy %.2f  clk %.2f GHz" % (k, names[k], dur, acc, req, acc / (cyc * 256) if cyc else 0, td / cyc if cyc else 0, cyc / dur / 1e6 if dur else 0))
