"""Headline benchmark: hammer-v0 env-steps/s on N MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs-per-gpu E]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" = one env-step of every env on every GPU: i.i.d. U(-1,1) actions from Philox
(seed 0, counter (env, step)), 5 physics substeps (frame_skip) + reward + obs, auto-reset at
the 200-step horizon inside the timed region, and at every episode boundary an RCCL all-gather
of the per-env episode returns / goal counts over xGMI.  Weak scaling: envs per GPU fixed
(default 65 536 = the north-star configuration).  Inputs are resident in HBM; value is
whole-job env-steps/s = N * envs_per_gpu * K / max-over-ranks wall time.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

ENV_ID = "hammer-v0"


def cpu_baseline(model_blob, env_id, budget_s=12.0):
    """Oracle (fp64 restatement, OpenMP over envs) on the host cores: bounded sample, all cores
    (2/3 of the budget) and one core (1/3), BASELINE.md §2."""
    import numpy as np
    from mj_envs_amd.tasks import attach_task, load_model, sample_params
    from oracle.pyoracle import Oracle, build
    build()
    m = attach_task(load_model(env_id), env_id)
    o = Oracle(model_blob)
    o.set_option(max_con=32, max_efc=128)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    threads = max(1, min(threads, 16))

    def run(nth, budget):
        n = 64 * nth
        rng = np.random.default_rng(0)
        P = sample_params(env_id, m, rng, n)
        st, _ = o.reset(P, nthreads=nth)
        steps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget:
            o.step(st, rng.uniform(-1, 1, (n, o.nu)), nthreads=nth)
            steps += 1
        dt = time.perf_counter() - t0
        return n * steps / dt, n, steps, dt

    v, n, steps, dt = run(threads, budget_s * 2 / 3)
    v1, n1, steps1, dt1 = run(1, budget_s / 3)
    return dict(value=v, unit="env-steps/s", cores=threads, kind="port",
                single_core_value=v1,
                sample=f"{env_id}, {n} envs x {steps} env-steps (random policy) on {threads} threads in {dt:.1f} s "
                       f"and {n1} envs x {steps1} env-steps on 1 thread in {dt1:.1f} s; fp64 C++ oracle "
                       f"(restated mj_step + task layer), OpenMP over envs")


def config2(blob, env_id, device, n=4096, steps=100, warmup=10):
    """BASELINE configs[1] (hammer-v0, 4 096 envs, random policy) as an auxiliary figure."""
    import torch
    from mj_envs_amd import _native
    sim = _native.Sim(blob, n, device=device)
    obs, act = sim.empty(n, sim.obs_dim), sim.empty(n, sim.nu)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    sim.reset(obs, seed=7)
    for k in range(warmup + steps):
        if k == warmup:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        sim.random_actions(act, 0, k)
        sim.step(act, obs, rew, done, goal, autoreset=True, seed=7)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sim.close()
    return dict(value=round(n * steps / dt, 1), unit="env-steps/s", envs=n, steps=steps,
                ms_per_step=round(dt / steps * 1e3, 4))


def pmc_traffic(env_per_launch):
    """HBM bytes per k_step launch from the committed rocprofv3 --pmc summary, or None."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_kstep.json")))
    if not paths:
        return None
    path = paths[-1]                         # latest round's counters
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("envs") != env_per_launch:
            return None
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs-per-gpu", type=int, default=65536)
    ap.add_argument("--total-envs", type=int, default=0,
                    help="strong scaling: fixed total envs split over the ranks (e.g. 262144, SURVEY C4)")
    ap.add_argument("--env", default=ENV_ID)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config2", action="store_true",
                    help="skip the auxiliary 4 096-env figure (profiling runs: every k_step launch is then "
                         "the headline size, so rocprof's average matches roofline.kernel_ms)")
    ap.add_argument("--policy", action="store_true",
                    help="closed loop: actions from the on-device Gaussian MLP (mjrl MLP, 32x32) instead of i.i.d.")
    ap.add_argument("--mpr", choices=("task", "fp32", "fp64"), default="task",
                    help="precision of the MPR (cylinder) collider: the task's default (tasks.py "
                         "TaskSpec.mpr_fp64; hammer fp32), or forced")
    ap.add_argument("--depth", action="store_true",
                    help="BASELINE config 5: + 64x64 depth-camera obs every env-step (default 8192 envs)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from mj_envs_amd import _native, perfmodel
    from mj_envs_amd.dist import EpisodeGather, rank_seed, shard_from_env
    from mj_envs_amd.tasks import TASKS, attach_task, load_model

    if args.depth and args.envs_per_gpu == 65536:
        args.envs_per_gpu = 8192
    if args.total_envs:
        w = int(os.environ.get("WORLD_SIZE", "1"))
        if args.total_envs % w:
            raise SystemExit("--total-envs must divide evenly over the ranks")
        args.envs_per_gpu = args.total_envs // w
    shard = shard_from_env(args.envs_per_gpu)
    world, rank, local = shard.world, shard.rank, shard.local_rank
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    env_id = args.env
    m = attach_task(load_model(env_id), env_id)
    blob = m.to_blob()
    n = args.envs_per_gpu
    sim = _native.Sim(blob, n, device=local)
    if args.mpr != "task":
        sim.set_option(disableflags=_native.DSBL_MPR_FP64 if args.mpr == "fp32" else _native.DSBL_MPR_FP32)
    mpr64 = args.mpr == "fp64" or (args.mpr == "task" and TASKS[env_id].mpr_fp64)
    obs = sim.empty(n, sim.obs_dim)
    act = sim.empty(n, sim.nu)
    rew = sim.empty(n)
    done = sim.empty(n, dtype=torch.uint8)
    goal = sim.empty(n, dtype=torch.uint8)
    last_ret = sim.empty(n)
    last_goal = sim.empty(n, dtype=torch.int32)
    gather = EpisodeGather(n, world, dev)
    seed = rank_seed(1, rank)                # per-rank Philox key: global env id = (rank, env)
    sim.reset(obs, seed=seed)
    pol = None
    if args.policy:
        from mj_envs_amd.policy import GaussianMLP
        pol = GaussianMLP(sim.obs_dim, sim.nu, (32, 32), init_log_std=-1.0, seed=0, device=local)
    depth = cam = None
    if args.depth:
        from mj_envs_amd.render import free_camera
        cam = free_camera(m, env_id, 64, 64)
        depth = sim.empty(n, 64, 64)

    def one_step(k, ev=None):
        if pol is not None:
            pol.act(obs, out=act, sample=True, seed=1000 * rank, step=k)
        else:
            sim.random_actions(act, 1000 * rank, k)
        if ev is not None:
            ev[0].record()
        sim.step(act, obs, rew, done, goal, autoreset=True, seed=seed)
        if ev is not None:
            ev[1].record()
        if depth is not None:
            if ev is not None:
                ev[2].record()
            sim.render_depth(depth, cam)
            if ev is not None:
                ev[3].record()
        if (k + 1) % sim.horizon == 0:       # every env finished an episode this step
            sim.episode_stats(last_ret, last_goal)
            gather(last_ret, last_goal)      # RCCL all-gather over xGMI when world > 1

    for k in range(args.warmup):
        one_step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    events = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(args.warmup + k, events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps
    depth_ms = sum(e[2].elapsed_time(e[3]) for e in events) / args.steps if depth is not None else None
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    finite = bool(torch.isfinite(obs).all())

    if rank == 0:
        total_steps = world * n * args.steps
        value = total_steps / elapsed
        flops, counts = perfmodel.step_flops(env_id, m, sim.frame_skip)
        achieved = flops * n / (kern_ms * 1e-3) / 1e12
        bytes_step = perfmodel.step_bytes(sim.nq, sim.nv, sim.nu, sim.obs_dim, sim.nparam)
        traffic = pmc_traffic(n)
        roof = dict(bound="mfma", achieved=round(achieved, 3), peak=perfmodel.PEAK_FP32_TFLOPS,
                    unit="TFLOP/s", frac=round(achieved / perfmodel.PEAK_FP32_TFLOPS, 5), traffic=traffic,
                    kernel=f"k_step<{sim.nv}>", kernel_ms=round(kern_ms, 4),
                    flops_per_env_step=round(flops), bytes_per_env_step=bytes_step,
                    hbm_achieved_GBps=round(bytes_step * n / (kern_ms * 1e-3) / 1e9, 2),
                    hbm_frac=round(bytes_step * n / (kern_ms * 1e-3) / 1e9 / perfmodel.PEAK_HBM_GBPS, 6),
                    note="fp32 compute roofline (VALU == f32 MFMA peak on gfx950); FLOPs from "
                         "perfmodel.py on profiles/work_counts_hammer.json")
        workload = (f"{env_id}, {n} envs per GPU (north-star config), random policy, auto-reset at horizon "
                    f"{sim.horizon}, RCCL all-gather of episode returns at episode ends")
        if pol is not None:
            workload = workload.replace("random policy", "closed loop with the on-device Gaussian MLP policy "
                                        "(mjrl MLP 32x32, random init, sampled actions)")
        if depth is not None:
            workload = (f"{env_id} + 64x64 depth-camera obs (HIP ray caster, BASELINE config 5), {n} envs per "
                        f"GPU, random policy, auto-reset at horizon {sim.horizon}")
            roof["depth_kernel_ms"] = round(depth_ms, 4)
        workload += ", MPR collider in " + ("fp64" if mpr64 else "fp32")
        metric = "env-steps/sec at N parallel envs, hammer-v0, 1/2/4/8 MI355X"
        if env_id != "hammer-v0":   # BASELINE config 3 lines are labelled with their own task
            metric = f"env-steps/sec at N parallel envs, {env_id}, 1/2/4/8 MI355X"
        line = dict(metric=metric,
                    value=round(value, 1), unit="env-steps/s", n_gpus=world, steps=args.steps,
                    warmup=args.warmup, ms_per_step=round(elapsed / args.steps * 1e3, 4),
                    higher_is_better=True, scaling="strong" if args.total_envs else "weak", vs_baseline=None,
                    dtype="f32",
                    data="synthetic (Philox U(-1,1) actions, reference reset distribution)",
                    config=dict(workload=workload, envs_per_gpu=n, total_envs=world * n,
                                frame_skip=sim.frame_skip, parallelism=f"env-shard x{world}"),
                    roofline=roof, finite=finite)
        if world == 1 and env_id == ENV_ID and depth is None and pol is None and n == 65536 and args.mpr == "task" \
                and not args.no_config2:
            line["config2_4096_envs"] = config2(blob, env_id, local)
        if world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(blob, env_id)
            except Exception as e:  # the baseline must not hide the GPU number
                line["cpu_baseline"] = dict(value=None, error=str(e))
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
