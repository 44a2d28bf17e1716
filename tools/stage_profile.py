"""Per-stage cycle breakdown of k_step (diagnostic build with -DAW_STAGE_PROF).

    python tools/stage_profile.py --build          # here: compile mj_envs_amd/libadroit_hip_prof.so
    python tools/stage_profile.py [--envs N] [--steps K] [--env hammer-v0]   # on the GPU box

Cycles are s_memtime shader-clock ticks per wave, summed over waves; the report divides by
the substep count to give cycles per wave-substep per stage.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF_LIB = os.path.join(REPO, "mj_envs_amd", "libadroit_hip_prof.so")


def build(task: int = 0):
    """one-TU profiling build of the fast tier + the task's wide-tier object (no markers there)"""
    sys.path.insert(0, REPO)
    from __graft_entry__ import HIPCC_FLAGS, compile_units, hipcc_path, wide_unit
    objdir = os.path.join(REPO, "build", "hip")
    os.makedirs(objdir, exist_ok=True)
    prof_o = os.path.join(objdir, "prof_fast.o")
    units = [(f"-DAW_STAGE_PROF -DAW_ONLY_TASK={task}", prof_o), wide_unit(task, objdir, "prof")]
    compile_units(units)
    subprocess.run([hipcc_path(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", PROF_LIB,
                    *[u[1] for u in units]], check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--env", default="hammer-v0")
    ap.add_argument("--out", default=None)
    ap.add_argument("--preroll", type=int, default=-1, help="untimed steps first (default: one horizon)")
    ap.add_argument("--policy", choices=("random", "dapg"), default="random",
                    help="actions: Philox U(-1,1) (the bench), or the reference's pretrained DAPG policy "
                         "(mean action, grasp regime)")
    a = ap.parse_args()
    if a.build:
        sys.path.insert(0, REPO)
        from mj_envs_amd.tasks import TASKS
        build(TASKS[a.env].kind)
        return
    os.environ["AW_LIB"] = PROF_LIB
    sys.path.insert(0, REPO)
    import torch
    from mj_envs_amd import _native
    from mj_envs_amd.tasks import attach_task, load_model
    m = attach_task(load_model(a.env), a.env)
    sim = _native.Sim(m.to_blob(), a.envs)
    obs = sim.empty(a.envs, sim.obs_dim)
    act = sim.empty(a.envs, sim.nu)
    rew, done, goal = sim.empty(a.envs), sim.empty(a.envs, dtype=torch.uint8), sim.empty(a.envs, dtype=torch.uint8)
    sim.reset(obs, seed=1)
    # the bench's steady state: staggered episode phases + one horizon of pre-roll
    from mj_envs_amd.dist import stagger_phases
    sim.set_episode(ep_len=torch.from_numpy(stagger_phases(a.envs, 0, sim.horizon)).cuda())
    pre = sim.horizon if a.preroll < 0 else a.preroll
    pol = None
    if a.policy == "dapg":
        from mj_envs_amd.policy import GaussianMLP
        pol = GaussianMLP.from_npz(os.path.join(REPO, "tests", "golden", f"dapg_{a.env.split('-')[0]}.npz"))

    def actions(k):
        if pol is not None:
            pol.act(obs, out=act)
        else:
            sim.random_actions(act, 0, k)

    for k in range(pre):
        actions(k)
        sim.step(act, obs, rew, done, goal, autoreset=True, seed=1)
    torch.cuda.synchronize()
    _native.stage_profile(reset=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for k in range(a.steps):
        actions(pre + k)
        sim.step(act, obs, rew, done, goal, autoreset=True, seed=1)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / a.steps
    p = _native.stage_profile(reset=True)
    sub = max(1, p["substeps"])
    names = _native.STAGES + _native.SUBSTAGES + _native.EXTRA_STAGES
    tot = sum(p[k] for k in names)
    rows = {k: dict(cycles_per_wave_substep=round(p[k] / sub, 1), frac=round(p[k] / max(tot, 1), 4))
            for k in names}
    res = dict(env=a.env, policy=a.policy, envs=a.envs, steps=a.steps, ms_per_step=round(ms, 3), waves=p["waves"],
               substeps=p["substeps"], cycles_per_wave_substep=round(tot / sub, 1), stages=rows,
               avg_newton_iters_per_solve=round(p["newton_iters"] / sub, 3),
               avg_noslip_iters_per_substep=round(p["noslip_iters"] / sub, 3),
               avg_nefc=round(p["nefc"] / sub, 3), avg_ncon=round(p["ncon"] / sub, 3),
               avg_offd_rows=round(p["offd_rows"] / sub, 3),
               avg_mpr_pairs=round(p["mpr_pairs"] / sub, 4), avg_mpr_contacts=round(p["mpr_contacts"] / sub, 4))
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
