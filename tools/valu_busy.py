"""VALU issue occupancy per kernel from a packaged profile (tools/package_profiles.sh): the
SQ_ACTIVE_INST_VALU pass (pmc_SQ_ACTIVE_INST_VALU_summary.csv) and the SQ_WAVE_CYCLES pass.

  valu_busy  = SQ_ACTIVE_INST_VALU * 4 / (CUs * 4 SIMDs) / (GRBM_GUI_ACTIVE / 8)
               (quad-cycles; GRBM_GUI_ACTIVE summed over the 8 XCDs: MI355X_MICROARCH.md) -- rocprof's
               VALUBusy with the SIMD count made explicit: the share of SIMD cycles with a VALU instruction
               of some wave in execution
  lane_util  = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64)   (active lanes per VALU cycle)
  valu_per_wave = SQ_INSTS_VALU / SQ_WAVES, wait_any = SQ_WAIT_ANY / SQ_WAVE_CYCLES (SQ_WAVE_CYCLES pass)
usage: valu_busy.py PROFILE_DIR [CUS]"""
import csv
import sys

d = sys.argv[1]
cus = int(sys.argv[2]) if len(sys.argv) > 2 else 256


def load(name):
    out = {}
    try:
        for r in csv.DictReader(open(f"{d}/{name}")):
            out.setdefault(r["kernel"], {})[r["counter"]] = (float(r["total"]), int(r["dispatches"]))
    except OSError:
        pass
    return out


v = load("pmc_SQ_ACTIVE_INST_VALU_summary.csv")
w = load("pmc_SQ_WAVE_CYCLES_summary.csv")
print(f"{'kernel':42s} {'disp':>5s} {'valu_busy':>9s} {'lane_util':>9s} {'valu/wave':>9s} {'wait_any':>8s} {'f64flop/valu':>12s}")
for k, c in sorted(v.items(), key=lambda kv: -kv[1].get("SQ_ACTIVE_INST_VALU", (0, 0))[0]):
    if "SQ_ACTIVE_INST_VALU" not in c or "GRBM_GUI_ACTIVE" not in c:
        continue
    act, n = c["SQ_ACTIVE_INST_VALU"]
    gui, _ = c["GRBM_GUI_ACTIVE"]
    thr, _ = c.get("SQ_THREAD_CYCLES_VALU", (0, 1))
    busy = act * 4 / (cus * 4) / (gui / 8) if gui else 0.0
    lane = thr / (act * 64) if act else 0.0
    ww = w.get(k, {})
    vpw = ww["SQ_INSTS_VALU"][0] / ww["SQ_WAVES"][0] if "SQ_INSTS_VALU" in ww and ww.get("SQ_WAVES", (0,))[0] else float("nan")
    wait = ww["SQ_WAIT_ANY"][0] / ww["SQ_WAVE_CYCLES"][0] if "SQ_WAIT_ANY" in ww and ww.get("SQ_WAVE_CYCLES", (0,))[0] else float("nan")
    f64 = c.get("SQ_INSTS_VALU_FLOPS_FP64", (0, 1))[0]
    ins = ww.get("SQ_INSTS_VALU", (0, 1))[0]
    print(f"{k[:42]:42s} {n:5d} {busy:9.3f} {lane:9.3f} {vpw:9.0f} {wait:8.3f} {(f64 / ins if ins else float('nan')):12.3f}")
