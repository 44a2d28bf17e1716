"""The measurement tooling's arithmetic (tools/summarize_profiles.py) on synthetic counter files:
the SQ_INST_LEVEL calibration (unit = chain latency x INSTS / LEVEL per class, applied to k_step's
counters) and the FETCH / WRITE calibration of the PMC summary (bytes / counter-to-exact ratio)."""
import csv
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def _csv(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Grid_Size",
                                          "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
                                          "SGPR_Count"])
        w.writeheader()
        for r in rows:
            w.writerow(dict(dict(Grid_Size=131072, Workgroup_Size=64, LDS_Block_Size=20480, Scratch_Size=132,
                                 VGPR_Count=128, SGPR_Count=112), **r))


def test_waitlvl_calibration(tmp_path, monkeypatch):
    import summarize_profiles as sp
    monkeypatch.setattr(sp, "REPO", str(tmp_path))
    os.makedirs(tmp_path / "profiles")
    src = tmp_path / "gpurun_out" / "t"
    # chains: latency L cycles per instruction, LEVEL = INSTS * L / unit with units 100 / 50 / 80
    lat = dict(lds=60.0, smem=64.0, vmem=160.0)
    unit = dict(lds=100.0, smem=50.0, vmem=80.0)
    os.makedirs(src)
    with open(src / "wl_cal.log", "w") as f:
        for c, v in lat.items():
            f.write(json.dumps(dict(chain=c, iters=4096, cycles_per_inst=v)) + "\n")
    rows = []
    for c, kern in (("lds", "k_lds_chain"), ("smem", "k_smem_chain"), ("vmem", "k_vmem_chain")):
        rows.append(dict(Dispatch_Id=1, Kernel_Name=kern, Counter_Name=f"SQ_INSTS_{c.upper()}", Counter_Value=1000))
        rows.append(dict(Dispatch_Id=1, Kernel_Name=kern, Counter_Name=f"SQ_INST_LEVEL_{c.upper()}",
                         Counter_Value=1000 * lat[c] / unit[c]))
    _csv(str(src / "wl_cal" / "wl_counter_collection.csv"), rows)
    # k_step: 2048 waves, 65 536 envs x 5 substeps -> 160 wave-substeps per wave
    waves, subs = 2048, 160
    k = [dict(Dispatch_Id=7, Kernel_Name="k_step<0>", Counter_Name="SQ_WAVES", Counter_Value=waves),
         dict(Dispatch_Id=7, Kernel_Name="k_step<0>", Counter_Name="SQ_WAVE_CYCLES", Counter_Value=waves * subs * 1000)]
    for c in ("lds", "smem", "vmem"):
        k.append(dict(Dispatch_Id=7, Kernel_Name="k_step<0>", Counter_Name=f"SQ_INSTS_{c.upper()}",
                      Counter_Value=waves * subs * 10))
        # each instruction outstanding 2 x the chain latency
        k.append(dict(Dispatch_Id=7, Kernel_Name="k_step<0>", Counter_Name=f"SQ_INST_LEVEL_{c.upper()}",
                      Counter_Value=waves * subs * 10 * 2 * lat[c] / unit[c]))
    _csv(str(src / "wl_kstep" / "wl_counter_collection.csv"), k)
    k2 = [dict(Dispatch_Id=7, Kernel_Name="k_step<0>", Counter_Name=n, Counter_Value=v) for n, v in (
        ("SQ_WAVES", waves), ("SQ_WAVE_CYCLES", waves * subs * 1000), ("SQ_WAIT_ANY", waves * subs * 400),
        ("SQ_WAIT_INST_ANY", waves * subs * 100), ("SQ_ACTIVE_INST_ANY", waves * subs * 500),
        ("SQ_ACTIVE_INST_VALU", waves * subs * 300), ("SQ_INSTS_VALU", waves * subs * 300),
        ("SQ_INSTS_SALU", waves * subs * 60))]
    _csv(str(src / "wl_kstep2" / "wl_counter_collection.csv"), k2)
    out = sp.waitlvl("t")
    for c in ("lds", "smem", "vmem"):
        assert out["calibration"][c]["cycles_per_level_unit"] == pytest.approx(unit[c])
        assert out["by_class"][c]["avg_latency_cycles"] == pytest.approx(2 * lat[c], rel=1e-3)
        assert out["by_class"][c]["frac_of_wave_life"] == pytest.approx(10 * 2 * lat[c] / 4000, rel=1e-3)
    assert out["wait_any_frac"] == pytest.approx(0.4)
    assert os.path.exists(tmp_path / "profiles" / "t_waitlvl_kstep.json")


def test_kernel_name_match_excludes_wide_tier():
    """k_step's counters must not absorb the wide tier's drain kernel (k_step_wide launches after
    every k_step, usually on an empty queue) or the profiling TU's variants"""
    import summarize_profiles as sp
    assert sp.is_kernel("void aw::fast128::k_step<0>(aw::DModel, float*)", "k_step")
    assert sp.is_kernel("k_step<2>", "k_step")
    assert not sp.is_kernel("void aw::wide::k_step_wide<0>(aw::DModel, float*)", "k_step")
    assert sp.is_kernel("k_step_wide<0>", "k_step_wide")
    assert sp.is_kernel("k_random_actions(float*, int)", "k_random_actions")
