"""Copy the judged parts of a gpurun_out/<tag> pass (tools/gpu_pass.sh + tools/gpu_prof.sh) into profiles/.

    python tools/summarize_profiles.py r01

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary),
profiles/<tag>_pmc_kstep.json (FETCH_SIZE / WRITE_SIZE of every k_step launch, per launch),
profiles/<tag>_bench.json (the bench line of the same pass) and profiles/<tag>_pytest_gpu.txt.
"""
import csv
import json
import re
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def is_kernel(name, kernel):
    """token match on the kernel name: "k_step" matches k_step<0>(...) but not k_step_wide<0>(...)
    (the wide tier's persistent drain kernel launches after every k_step, usually on an empty queue)"""
    return re.search(r"\b" + re.escape(kernel) + r"(?![A-Za-z0-9_])", name) is not None


def pmc(path, counter, kernel="k_step"):
    vals, meta = [], {}
    for r in csv.DictReader(open(path)):
        if is_kernel(r["Kernel_Name"], kernel) and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
            meta = dict(grid=int(r["Grid_Size"]), wg=int(r["Workgroup_Size"]), lds=int(r["LDS_Block_Size"]),
                        scratch=int(r["Scratch_Size"]), vgpr=int(r["VGPR_Count"]), sgpr=int(r["SGPR_Count"]),
                        name=r["Kernel_Name"])
    return vals, meta


def last_json(path):
    """the last JSON line a bench run printed (None if the file is absent or has none)"""
    if not os.path.exists(path):
        return None
    for ln in reversed(open(path).read().splitlines()):
        if ln.startswith("{"):
            return json.loads(ln)
    return None


def main(tag):
    src = os.path.join(REPO, "gpurun_out", tag)
    dst = os.path.join(REPO, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "kt_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    bench = open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1]
    b = json.loads(bench)
    with open(os.path.join(dst, f"{tag}_bench.json"), "w") as f:
        f.write(bench + "\n")
    log = os.path.join(src, "pytest_gpu.log")
    if os.path.exists(log):
        shutil.copy(log, os.path.join(dst, f"{tag}_pytest_gpu.txt"))
    fetch, meta = pmc(os.path.join(src, "pmc_fetch", "pf_counter_collection.csv"), "FETCH_SIZE")
    write, _ = pmc(os.path.join(src, "pmc_write", "pw_counter_collection.csv"), "WRITE_SIZE")
    # calibration kernel on the same box: k_random_actions writes exactly n*nu*4 bytes
    cal, _ = pmc(os.path.join(src, "pmc_write", "pw_counter_collection.csv"), "WRITE_SIZE", "k_random_actions")
    # persistent k_step workgroups: the grid is the resident-slot count, not the env count
    # the run identity comes from the bench line the PMC pass itself printed (falls back to the
    # pass's bench.json); bench.py's pmc_traffic only reports a summary whose identity matches
    pb = last_json(os.path.join(src, "pmc_fetch.log")) or b
    envs = pb["config"].get("envs_per_gpu", meta["grid"] // meta["wg"])
    fetch_b = statistics.mean(fetch) * 1024
    write_b = statistics.mean(write) * 1024
    nu = 26 if "hammer" in pb["config"]["workload"] else None
    # counter calibration on the same box (tools/mb/calib.hip: one wave per 132-byte row, 4 B per
    # lane -- k_step's state / obs pattern -- with exactly known bytes): counter / exact per direction
    cal_pat = None
    cf = os.path.join(src, "cal_fetch", "cf_counter_collection.csv")
    cw = os.path.join(src, "cal_write", "cw_counter_collection.csv")
    if os.path.exists(cf) and os.path.exists(cw):
        ex = last_json(os.path.join(src, "cal_fetch.log"))
        f_c, _ = pmc(cf, "FETCH_SIZE", "k_calib_read")
        w_c, _ = pmc(cw, "WRITE_SIZE", "k_calib_write")
        cal_pat = dict(kernels="tools/mb/calib.hip k_calib_read / k_calib_write",
                       exact_read_bytes=ex["exact_read_bytes"], exact_write_bytes=ex["exact_write_bytes"],
                       fetch_ratio=round(statistics.mean(f_c) * 1024 / ex["exact_read_bytes"], 4),
                       write_ratio=round(statistics.mean(w_c) * 1024 / ex["exact_write_bytes"], 4))
    out = dict(
        tag=tag, kernel=meta["name"], envs=envs, launches=len(fetch),
        env_id=pb["config"].get("env_id"), policy=pb["config"].get("policy"),
        kernel_build_id=pb["roofline"].get("kernel_build_id"),
        fetch_size_kb=[round(v, 3) for v in fetch], write_size_kb=[round(v, 3) for v in write],
        fetch_bytes_per_launch=round(fetch_b), write_bytes_per_launch=round(write_b),
        hbm_bytes_per_launch=round(fetch_b + write_b),
        hbm_bytes_per_env_step=round((fetch_b + write_b) / envs, 1),
        algorithmic_bytes_per_env_step=b["roofline"]["bytes_per_env_step"],
        write_calibration=None if not cal or nu is None else dict(
            kernel="k_random_actions", exact_bytes=envs * nu * 4,
            write_size_bytes=round(statistics.mean(cal) * 1024),
            ratio=round(statistics.mean(cal) * 1024 / (envs * nu * 4), 3)),
        kernel_resources=dict((k, meta[k]) for k in ("wg", "lds", "scratch", "vgpr", "sgpr")),
        calibration=cal_pat,
        hbm_bytes_per_launch_calibrated=None if cal_pat is None else round(
            fetch_b / cal_pat["fetch_ratio"] + write_b / cal_pat["write_ratio"]),
        method="rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
               "`python bench.py --steps 3 --warmup 1 --no-cpu-baseline` (MI355X_MICROARCH.md HBM section); "
               "counters are KB (x1024). FETCH_SIZE is NOT doubled: the 1/2 tally the guide documents is for "
               "16 B/lane streaming reads, while k_step reads each env's state as one 4 B/lane row per wave "
               "(uncalibrated width); raw counter bytes are reported, and beside them the bytes divided by "
               "the same box's calibration for exactly that pattern (calibration).")
    with open(os.path.join(dst, f"{tag}_pmc_kstep.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("envs", "hbm_bytes_per_launch", "hbm_bytes_per_env_step",
                                          "algorithmic_bytes_per_env_step", "write_calibration",
                                          "calibration", "hbm_bytes_per_launch_calibrated")}))


def sq(tag):
    """SQ issue / wait split of k_step from the three --pmc passes of tools/gpu_prof.sh"""
    import collections
    src = os.path.join(REPO, "gpurun_out", tag)
    per = {}
    for f in ("sq1", "sq2", "sq3"):
        path = os.path.join(src, f, f"{f}_counter_collection.csv")
        if not os.path.exists(path):
            return None
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(path)):
            if is_kernel(r["Kernel_Name"], "k_step"):
                agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for c, d in agg.items():
            per[c] = sum(d.values()) / len(d)
    waves = per["SQ_WAVES"]
    subs = 65536 * 5 / waves          # wave-substeps per wave (headline launch: 65 536 envs x 5)
    wc = per["SQ_WAVE_CYCLES"]
    out = dict(tag=tag, kernel="k_step (hammer-v0, 65 536 envs, persistent grid)", per_dispatch=per,
               per_wave_substep={k: round(v / waves / subs, 1) for k, v in per.items() if k != "SQ_WAVES"},
               fractions_of_wave_cycles={k: round(per[c] / wc, 4) for k, c in (
                   ("active_inst_any", "SQ_ACTIVE_INST_ANY"), ("active_valu", "SQ_ACTIVE_INST_VALU"),
                   ("active_lds", "SQ_ACTIVE_INST_LDS"), ("wait_any", "SQ_WAIT_ANY"),
                   ("wait_inst_any", "SQ_WAIT_INST_ANY"), ("wait_inst_lds", "SQ_WAIT_INST_LDS"))},
               note="SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (x4 = shader cycles); "
                    "WAIT_ANY = parked on s_waitcnt, WAIT_INST_ANY = issue stall on a dependency, "
                    "ACTIVE_INST_ANY = issuing (MI355X_MICROARCH.md PMC section)")
    with open(os.path.join(REPO, "profiles", f"{tag}_sq_kstep.json"), "w") as f:
        json.dump(out, f, indent=1)
    return out


def waitlvl(tag):
    """k_step's s_waitcnt exposure split by instruction class (tools/gpu_waitlvl.sh): the
    SQ_INST_LEVEL_* counters (outstanding instructions accumulated over time, unit unknown) are
    scaled by dependent-chain kernels whose per-instruction latency s_memtime measures
    (tools/mb/waitlvl.hip): unit = latency x INSTS / LEVEL per class."""
    import collections
    src = os.path.join(REPO, "gpurun_out", tag)

    def agg(path, kern):
        a = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(path)):
            if is_kernel(r["Kernel_Name"], kern):
                a[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        return {c: sum(d.values()) / len(d) for c, d in a.items()}

    lat = {}
    for ln in open(os.path.join(src, "wl_cal.log")):
        if ln.startswith("{") and "chain" in ln:
            d = json.loads(ln)
            lat[d["chain"]] = d["cycles_per_inst"]
    cal_csv = os.path.join(src, "wl_cal", "wl_counter_collection.csv")
    unit = {}
    for cls, kern in (("lds", "k_lds_chain"), ("smem", "k_smem_chain"), ("vmem", "k_vmem_chain")):
        c = agg(cal_csv, kern)
        K = cls.upper()
        unit[cls] = dict(latency_cycles=lat[cls], insts=c[f"SQ_INSTS_{K}"], level=c[f"SQ_INST_LEVEL_{K}"],
                         cycles_per_level_unit=lat[cls] * c[f"SQ_INSTS_{K}"] / c[f"SQ_INST_LEVEL_{K}"])
    k = agg(os.path.join(src, "wl_kstep", "wl_counter_collection.csv"), "k_step")
    k2 = {}   # WAIT / ACTIVE / INSTS_VALU / SALU: tools/gpu_waitlvl.sh's second pass, or gpu_prof.sh's sq1 + sq2
    for f in (("wl_kstep2", "wl"), ("sq1", "sq1"), ("sq2", "sq2")):
        path = os.path.join(src, f[0], f"{f[1]}_counter_collection.csv")
        if os.path.exists(path):
            k2.update(agg(path, "k_step"))
    waves = k["SQ_WAVES"]
    subs = 65536 * 5 / waves
    life = k["SQ_WAVE_CYCLES"] * 4 / waves / subs          # shader cycles per wave-substep
    cls_out = {}
    for cls in ("lds", "smem", "vmem"):
        K = cls.upper()
        oc = k[f"SQ_INST_LEVEL_{K}"] * unit[cls]["cycles_per_level_unit"] / waves / subs
        cls_out[cls] = dict(insts_per_wave_substep=round(k[f"SQ_INSTS_{K}"] / waves / subs, 1),
                            avg_latency_cycles=round(oc / (k[f"SQ_INSTS_{K}"] / waves / subs), 1),
                            outstanding_cycles_per_wave_substep=round(oc),
                            frac_of_wave_life=round(oc / life, 4))
    out = dict(tag=tag, kernel="k_step (hammer-v0, 65 536 envs)", calibration=unit,
               wave_life_cycles_per_wave_substep=round(life),
               wait_any_frac=round(k2["SQ_WAIT_ANY"] / k2["SQ_WAVE_CYCLES"], 4),
               wait_inst_any_frac=round(k2["SQ_WAIT_INST_ANY"] / k2["SQ_WAVE_CYCLES"], 4),
               active_inst_any_frac=round(k2["SQ_ACTIVE_INST_ANY"] / k2["SQ_WAVE_CYCLES"], 4),
               active_valu_frac=round(k2["SQ_ACTIVE_INST_VALU"] / k2["SQ_WAVE_CYCLES"], 4),
               valu_per_wave_substep=round(k2["SQ_INSTS_VALU"] / k2["SQ_WAVES"] / (65536 * 5 / k2["SQ_WAVES"]), 1),
               salu_per_wave_substep=round(k2["SQ_INSTS_SALU"] / k2["SQ_WAVES"] / (65536 * 5 / k2["SQ_WAVES"]), 1),
               by_class=cls_out,
               note="outstanding cycles overlap (several loads in flight count several times) and overlap "
                    "the other wave's issue: they bound, not partition, the s_waitcnt time")
    with open(os.path.join(REPO, "profiles", f"{tag}_waitlvl_kstep.json"), "w") as f:
        json.dump(out, f, indent=1)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "waitlvl":
        print(json.dumps(waitlvl(sys.argv[2]), indent=1))
        sys.exit(0)
    t = sys.argv[1] if len(sys.argv) > 1 else "r01"
    main(t)
    r = sq(t)
    if r:
        print(json.dumps(r["fractions_of_wave_cycles"]))
    for f in ("stage_profile.json", "stage_profile_dapg.json"):
        p = os.path.join(REPO, "gpurun_out", t, f)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(REPO, "profiles", f"{t}_{f}"))
