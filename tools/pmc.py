#!/usr/bin/env python3
"""Collect rocprofv3 PMC counters for the record-engine kernels, one counter group per pass
(never combined with tracing), and summarise them per kernel.

Usage (on the GPU box, from the repo root):
    python tools/pmc.py --out gpurun_out/pmc --summary profiles/pmc_r01.json -- \
        python3 bench.py --no-cpu-baseline --steps 3 --warmup 1

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE (KiB) reads exactly half of a wide
coalesced streaming read on gfx950 and is doubled; WRITE_SIZE (KiB) is taken as is.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import subprocess
import sys

PASSES = [
    ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
     "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "GRBM_GUI_ACTIVE"],
    ["SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
     "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_INSTS_VMEM"],
    ["TA_BUSY_avr", "TD_TD_BUSY_sum", "VALUBusy", "GRBM_GUI_ACTIVE"],
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
]


# --passes stall: where the waves of the streaming kernel wait (issue stalls at the texture unit,
# FIFO-full cycles, L2-to-fabric credit stalls)
STALL_PASSES = [
    ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM",
     "SQ_INST_CYCLES_VMEM_RD", "SQ_INST_CYCLES_VMEM_WR", "SQ_ACTIVE_INST_ANY"],
    ["SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_VMEM_TA_CMD_FIFO_FULL", "SQ_VMEM_WR_TA_DATA_FIFO_FULL",
     "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_IFETCH", "SQ_BUSY_CYCLES",
     "TA_ADDR_STALLED_BY_TC_CYCLES", "TA_DATA_STALLED_BY_TC_CYCLES", "GRBM_GUI_ACTIVE"],
    ["TCC_EA0_WRREQ_STALL", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL", "TCC_EA0_WRREQ_DRAM_CREDIT_STALL",
     "GRBM_GUI_ACTIVE"],
]


def kernel_key(name: str):
    if not any(k in name for k in ("records_kernel", "sha_kernel", "stream_kernel", "duplex_kernel",
                                   "duplex_split_kernel", "seg_uniform", "seg_kernel", "seg_plan")):
        return None
    return name.split("(")[0].replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/pmc")
    ap.add_argument("--summary", default=None)
    ap.add_argument("--config", default=None, help="JSON dict recorded as the workload config")
    ap.add_argument("--passes", default="default", choices=["default", "stall", "traffic"])
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    os.makedirs(a.out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    sets = {"default": PASSES, "stall": STALL_PASSES, "traffic": [["FETCH_SIZE"], ["WRITE_SIZE"]]}
    for i, counters in enumerate(sets[a.passes]):
        tag = f"p{i}"
        rc = subprocess.run(["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d",
                             a.out, "-o", tag, "--", *cmd], env=env,
                            stdout=subprocess.DEVNULL, stderr=open(os.path.join(a.out, f"{tag}.err"), "w"),
                            timeout=600).returncode
        if rc != 0:
            print(f"pass {tag} failed rc={rc}", file=sys.stderr)
            sys.exit(rc)
        for f in glob.glob(os.path.join(a.out, "**", f"{tag}_counter_collection.csv"), recursive=True):
            seen = set()
            for row in csv.DictReader(open(f)):
                k = kernel_key(row["Kernel_Name"])
                if k:
                    vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    did = (row["Dispatch_Id"], tag)
                    if did not in seen:
                        seen.add(did)
                        dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                        vals[k][f"dur_ns_{tag}"].append(float(dur))
    summary = {"config": json.loads(a.config) if a.config else None, "kernels": {}}
    for k, d in vals.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        out = dict(m)
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            out["hbm_bytes_per_launch"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        if "GRBM_GUI_ACTIVE" in m and "dur_ns_p0" in m:
            out["eff_clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8.0 / m["dur_ns_p0"]
        if "GRBM_GUI_ACTIVE" in m and "SQ_ACTIVE_INST_VALU" in m:
            cyc = m["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
            # on gfx950 SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU (an instruction count summed over
            # the 1024 SIMDs, not busy cycles): report kernel cycles per VALU instruction per SIMD
            out["cycles_per_valu_instr_per_simd"] = cyc / (m["SQ_ACTIVE_INST_VALU"] / 1024.0)
            out["kernel_cycles"] = cyc
        if "TA_BUSY_avr" in m and "GRBM_GUI_ACTIVE" in m:
            out["ta_busy_frac"] = m["TA_BUSY_avr"] / (m["GRBM_GUI_ACTIVE"] / 8.0)
        summary["kernels"][k] = out
    txt = json.dumps(summary, indent=1, sort_keys=True)
    print(txt)
    if a.summary:
        os.makedirs(os.path.dirname(a.summary) or ".", exist_ok=True)
        with open(a.summary, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
