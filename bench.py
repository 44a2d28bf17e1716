"""Headline benchmark: hammer-v0 env-steps/s on N MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs-per-gpu E]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` outside torch.distributed.run starts N ranks itself (`dist.launch_ranks`: one child
process per GPU, RANK / LOCAL_RANK / WORLD_SIZE set, the parent never touches the GPU) and exits
non-zero when fewer than N devices are visible -- it never falls back to one GPU.  `--launch`
takes the same path at N = 1 (one rank, RCCL process group of one); `--dry-run` runs the launcher
and the episode-totals exchange over gloo with no GPU and no kernel (the CPU test of this path).

A "step" = one env-step of every env on every GPU: i.i.d. U(-1,1) actions from Philox (seed 0,
counter (global env id, step)), frame_skip = 5 physics substeps + reward + obs, and auto-reset
inside the kernel whenever an episode ends.  Episode phases are staggered (each env's first
episode starts at a hash of its global id modulo the horizon) and an untimed pre-roll of one
horizon runs before the warm-up, so every timed window is in steady state: ~N/200 envs end an
episode and reset on every step, and all episode phases are present.  Every `horizon` steps
(and at the end) the per-env totals over finished episodes (count, summed return, successes)
are all-gathered over RCCL / xGMI -- every finished episode is counted once, whenever it
ended.  Weak scaling: envs per GPU fixed (default 65 536 = the north-star configuration).
Inputs are resident in HBM; value = N * envs_per_gpu * K / max-over-ranks wall time.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

ENV_ID = "hammer-v0"
SEED_RESET, SEED_ACT = 1, 0


def cpu_threads():
    """Host threads available to this job: the CPU affinity mask, capped by OMP_NUM_THREADS (the
    GPU box grants 16 per GPU and sets it; nproc there reports the whole machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(omp)) if omp else aff), aff


def gpu_inputs(blob, n, steps, local):
    """The GPU run's own inputs for the first n envs: reset params (Philox, seed SEED_RESET,
    global env ids 0..n-1) and `steps` steps of actions (seed SEED_ACT), copied to the host."""
    import numpy as np
    import torch
    from mj_envs_amd import _native
    sim = _native.Sim(blob, n, device=local)
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, seed=SEED_RESET)
    p = sim.empty(n, sim.nparam)
    sim.get_state(params=p)
    act = sim.empty(steps, n, sim.nu)
    for k in range(steps):
        sim.random_actions(act[k], SEED_ACT, k)
    torch.cuda.synchronize()
    out = p.cpu().numpy().astype(np.float64), act.cpu().numpy().astype(np.float64)
    sim.close()
    return out


def cpu_baseline(blob, env_id, local, budget_s=12.0):
    """Oracle (fp64 restatement, OpenMP over envs) on the host cores, on the GPU run's own reset
    params and Philox actions: all available threads (2/3 of the budget) and one (1/3)."""
    from oracle.pyoracle import Oracle, build
    build()
    o = Oracle(blob)
    threads, aff = cpu_threads()

    def run(nth, budget):
        n = 64 * nth
        P, A = gpu_inputs(blob, n, 600, local)
        st, _ = o.reset(P, nthreads=nth)
        steps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget and steps < A.shape[0]:
            o.step(st, A[steps], nthreads=nth)
            steps += 1
        dt = time.perf_counter() - t0
        return n * steps / dt, n, steps, dt

    v, n, steps, dt = run(threads, budget_s * 2 / 3)
    v1, n1, steps1, dt1 = run(1, budget_s / 3)
    return dict(value=round(v, 1), unit="env-steps/s", cores=threads, kind="port",
                label="restated CPU reference (fp64 C++ oracle of the task layer + MuJoCo 2.1 mj_step)",
                single_core_value=round(v1, 1), nproc=os.cpu_count(), affinity_cpus=aff,
                omp_num_threads=os.environ.get("OMP_NUM_THREADS"),
                all_affinity_cpus_linear_estimate=round(v / threads * aff, 1),
                why_not_all_cpus=(f"the GPU box grants one GPU's job {threads} host threads (OMP_NUM_THREADS="
                                  f"{os.environ.get('OMP_NUM_THREADS')}; worker pools must stay within that "
                                  f"share) while its affinity mask shows all {aff} CPUs of the shared node; "
                                  f"all_affinity_cpus_linear_estimate scales the measured per-thread rate to "
                                  f"{aff} CPUs (an upper bound, not measured)") if aff > threads else None,
                sample=f"{env_id}, the GPU run's first {n} envs (its Philox reset params and actions) x {steps} "
                       f"env-steps on {threads} threads in {dt:.1f} s, and {n1} envs x {steps1} env-steps on 1 "
                       f"thread in {dt1:.1f} s; fp64 C++ oracle (restated mj_step + task layer at MuJoCo's "
                       f"capacities), OpenMP over envs; threads = the job's CPU share (affinity / OMP_NUM_THREADS)")


def _oracle_f32_model(m):
    """the fp64 oracle on the model the GPU holds (every float model constant rounded to fp32)"""
    import copy
    import numpy as np
    from oracle.pyoracle import Oracle
    m = copy.deepcopy(m)
    for k, v in list(m.arrays.items()):
        a = np.asarray(v)
        if a.dtype.kind == "f":
            m.arrays[k] = a.astype(np.float32).astype(np.float64)
    m.opt = {k: (float(np.float32(v)) if isinstance(v, float) else v) for k, v in m.opt.items()}
    return Oracle(m.to_blob())


def _miss_is_fp32_sensitive(o, o32, st, act, gpu=None, trials=8, ulps=16, seed=0, factor=4.0, ratio_out=None):
    """tests/parity_classify.py fp32_sensitive: the oracle's own env-step leaves the one-step
    tolerance when re-run on the fp32-rounded model or from the state perturbed by <= 16 fp32 ulps
    per component -- the step is on a switch / ill-conditioned at fp32 resolution -- AND (given the
    GPU's post-step state gpu = (qpos, qvel)) the GPU's deviation from the unperturbed fp64 result
    is within `factor` x the largest deviation of those runs (or within tolerance), in qpos and qvel.
    ratio_out (a list) receives the GPU's deviation / the runs' spread (0 where within tolerance),
    so a drift towards `factor` stays visible (advisor r05)"""
    import numpy as np
    rng = np.random.default_rng(seed)
    base = {k: v.copy() for k, v in st.items()}
    o.step(base, act)
    runs = [(o32, {k: v.copy() for k, v in st.items()})]
    eps = ulps * 2.0 ** -23
    for _ in range(trials):
        p = dict(params=st["params"].copy())
        for k in ("qpos", "qvel", "warm"):
            p[k] = st[k] * (1 + eps * rng.uniform(-1, 1, st[k].shape))
        runs.append((o, p))
    bq, bv = base["qpos"], base["qvel"]
    tolq = lambda q: (np.abs(q - bq) <= 2e-5 + 1e-5 * np.abs(bq)).all()
    tolv = lambda v: (np.abs(v - bv) <= 5e-3 * (1 + np.abs(bv))).all()
    leaves, dq, dv = False, 0.0, 0.0
    for oo, p in runs:
        oo.step(p, act)
        leaves |= not (tolq(p["qpos"]) and tolv(p["qvel"]))
        dq = max(dq, float(np.abs(p["qpos"] - bq).max()))
        dv = max(dv, float((np.abs(p["qvel"] - bv) / (1 + np.abs(bv))).max()))
    if not leaves or gpu is None:
        return leaves
    gq, gv = np.asarray(gpu[0], float).reshape(bq.shape), np.asarray(gpu[1], float).reshape(bv.shape)
    eq, ev = float(np.abs(gq - bq).max()), float((np.abs(gv - bv) / (1 + np.abs(bv))).max())
    rq = 0.0 if tolq(gq) else (eq / dq if dq > 0 else float("inf"))
    rv = 0.0 if tolv(gv) else (ev / dv if dv > 0 else float("inf"))
    if ratio_out is not None:
        ratio_out.append(max(rq, rv))
    return bool(rq <= factor and rv <= factor)


def same_run_parity(blob, sim, n=256, model=None, pol=None, obs_now=None):
    """One env-step of the benchmark's OWN handle (all its envs, the timed run's launch
    configuration: persistent workgroups claiming envs past the resident slots) from its mid-run
    states, checked on n envs sampled evenly across the whole batch against the fp64 oracle from
    the same pre-step states: fraction within the one-step tolerance of tests/test_gpu_parity.py
    and the errors.  Runs after the timed region (no auto-reset in this step)."""
    import numpy as np
    import torch
    from oracle.pyoracle import Oracle, build
    build()
    N = sim.n_envs
    q, v, w, p = sim.empty(N, sim.nq), sim.empty(N, sim.nv), sim.empty(N, sim.nv), sim.empty(N, sim.nparam)
    sim.get_state(q, v, w, p)
    act = sim.empty(N, sim.nu)
    if pol is not None and obs_now is not None:
        pol.act(obs_now, out=act)        # the closed loop's own (mean) action: the regime the bench timed
    else:
        sim.random_actions(act, 12345, 0)
    obs, rew = sim.empty(N, sim.obs_dim), sim.empty(N)
    done, goal = sim.empty(N, dtype=torch.uint8), sim.empty(N, dtype=torch.uint8)
    sim.step(act, obs, rew, done, goal)
    q2, v2 = sim.empty(N, sim.nq), sim.empty(N, sim.nv)
    sim.get_state(q2, v2)
    torch.cuda.synchronize()
    idx = np.unique(np.linspace(0, N - 1, min(n, N)).round().astype(int))
    g = lambda t: t.cpu().numpy()[idx].astype(np.float64)
    st = dict(qpos=g(q), qvel=g(v), warm=g(w), params=g(p))
    o = Oracle(blob)
    st0 = {k: v.copy() for k, v in st.items()}   # the pre-step states (o.step advances st in place)
    o_obs, o_rew, _, _, _ = o.step(st, g(act))
    qg, vg = q2.cpu().numpy()[idx], v2.cpu().numpy()[idx]
    okq = (np.abs(qg - st["qpos"]) <= 2e-5 + 1e-5 * np.abs(st["qpos"])).all(axis=1)
    okv = (np.abs(vg - st["qvel"]) <= 5e-3 * (1 + np.abs(st["qvel"]))).all(axis=1)
    ok = okq & okv
    # every miss re-checked as the parity tests do: is the fp64 reference itself unstable at fp32
    # resolution there, with the GPU inside that instability (tests/test_gpu_parity.py
    # _classify_misses, criterion b)?  All misses are classified.
    sens, ratios = [], []
    miss_idx = np.nonzero(~ok)[0]
    if model is not None and miss_idx.size:
        o32 = _oracle_f32_model(model)
        for k in miss_idx:
            stk = {key: st0[key][k:k + 1].copy() for key in st0}
            sens.append(bool(_miss_is_fp32_sensitive(o, o32, stk, g(act)[k:k + 1],
                                                     gpu=(qg[k:k + 1], vg[k:k + 1]), ratio_out=ratios)))
    eq = np.abs(qg - st["qpos"]).max(axis=1)
    ev = (np.abs(vg - st["qvel"]) / (1 + np.abs(st["qvel"]))).max(axis=1)
    return dict(envs=len(idx), handle_envs=N, grid=sim.grid, sampled="evenly over the whole batch (incl. "
                f"{int((idx >= sim.grid).sum())} envs past the {sim.grid} resident slots)",
                frac_within_tol=round(float(ok.mean()), 4), misses=[int(i) for i in idx[~ok]],
                misses_classified=len(sens) if model is not None else 0,
                misses_fp32_sensitive_reference=sum(sens), misses_unexplained=len(sens) - sum(sens)
                if model is not None else None,
                miss_spread_ratios=[round(r, 3) for r in ratios], max_spread_ratio=max(ratios) if ratios else None,
                max_abs_qpos=float(eq.max()), max_rel_qvel=float(ev.max()),
                p50_abs_qpos=float(np.median(eq)), p99_abs_qpos=float(np.percentile(eq, 99)),
                median_abs_obs=float(np.median(np.abs(obs.cpu().numpy()[idx] - o_obs))),
                max_abs_reward=float(np.abs(rew.cpu().numpy()[idx] - o_rew).max()),
                tolerance="qpos 2e-5 + 1e-5|q|, qvel 5e-3 (1 + |v|) per env (tests/test_gpu_parity.py)")


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


def pmc_traffic(envs, env_id, policy, build_id):
    """HBM bytes per k_step launch (raw, calibrated, source, calibration) from the newest committed
    rocprofv3 --pmc summary whose run matches this one exactly -- env count, task, policy and the
    kernel build id (hash of the HIP sources + flags) -- or (None, None, None): a summary of another
    workload or another kernel revision is never reported as this run's traffic."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_kstep.json")), reverse=True)
    for path in paths:
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if (d.get("envs"), d.get("env_id"), d.get("policy"), d.get("kernel_build_id")) == \
                (envs, env_id, policy, build_id):
            return (d.get("hbm_bytes_per_launch"), d.get("hbm_bytes_per_launch_calibrated"),
                    os.path.relpath(path, REPO), d.get("calibration"))
    return None, None, None, None


def dry_run(args, shard):
    """The launcher's CPU rehearsal: each rank joins a gloo group, fills its block of the packed
    episode-totals buffer with rank-specific values (env i of the global batch finished i % 3
    episodes with return i each, successes on odd global ids) and does the one all-gather bench.py
    does every horizon; rank 0 prints one JSON line with every rank's shard and the exchange."""
    import torch
    import torch.distributed as dist
    from mj_envs_amd.dist import EpisodeTotals, under_launcher
    if under_launcher():
        dist.init_process_group("gloo")
    n, off = shard.envs_per_rank, shard.env_offset
    totals = EpisodeTotals(n, shard.world, "cpu")
    ep, ret, suc = totals.rows()
    gid = torch.arange(off, off + n)
    ep.copy_(gid % 3)
    ret.copy_((gid % 3).float() * gid.float())
    suc.copy_((gid % 3) * (gid % 2))
    e, r, s = totals()
    me = dict(rank=shard.rank, local_rank=shard.local_rank, world=shard.world, env_offset=off, envs=n,
              pid=os.getpid())
    ranks = [None] * shard.world
    if dist.is_initialized():
        dist.all_gather_object(ranks, me)
    else:
        ranks = [me]
    if shard.rank == 0:
        gexp = torch.arange(shard.world * n)
        line = dict(dry_run=True, n_gpus=shard.world, ranks=ranks,
                    config=dict(parallelism=f"env-shard x{shard.world}", envs_per_gpu=n, total_envs=shard.total_envs),
                    exchange=dict(backend=dist.get_backend() if dist.is_initialized() else "local copy",
                                  calls=totals.calls, bytes_per_rank_per_call=totals.bytes_per_rank,
                                  episodes_ok=bool(torch.equal(e.long(), gexp % 3)),
                                  returns_ok=bool(torch.equal(r, ((gexp % 3) * gexp).float())),
                                  successes_ok=bool(torch.equal(s.long(), (gexp % 3) * (gexp % 2))),
                                  summary=totals.summary()))
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def default_preroll(horizon, warmup, steps):
    """untimed pre-roll: at least one horizon (steady state: every env past its staggered first episode),
    extended so that the timed window [preroll + warmup, preroll + warmup + steps) holds a horizon
    boundary -- step k with (k + 1) % horizon == 0, where the episode totals are all-gathered -- near
    its middle: any --steps >= 1 times one exchange (the collective is part of the timed workload)"""
    t = max(1, steps // 2)
    return horizon + (-(warmup + t)) % horizon


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--preroll", type=int, default=-1,
                    help="untimed steps after the staggered reset (default: one horizon plus the offset that "
                         "puts a horizon boundary -- the episode-totals exchange -- inside the timed window), "
                         "so the timed window starts in steady state")
    ap.add_argument("--envs-per-gpu", type=int, default=65536)
    ap.add_argument("--total-envs", type=int, default=0,
                    help="strong scaling: fixed total envs split over the ranks (e.g. 262144, SURVEY C4)")
    ap.add_argument("--env", default=ENV_ID)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-config2", action="store_true",
                    help="skip the auxiliary 4 096-env figure (profiling runs: every k_step launch is then "
                         "the headline size, so rocprof's average matches roofline.kernel_ms)")
    ap.add_argument("--policy", choices=("none", "random-mlp", "dapg"), default="none",
                    help="closed loop: actions from the on-device Gaussian MLP (k_mlp): random init 32x32 "
                         "(sampled), or the reference's pretrained DAPG policy (mean action)")
    ap.add_argument("--depth", action="store_true",
                    help="BASELINE config 5: + 64x64 depth-camera obs every env-step (default 8192 envs)")
    ap.add_argument("--launch", action="store_true",
                    help="start the ranks through the launcher even for --gpus 1 (one-rank RCCL group)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + episode-totals exchange over gloo, no GPU, no kernel (CPU test)")
    args = ap.parse_args()

    from mj_envs_amd.dist import EpisodeTotals, launch_ranks, shard_from_env, stagger_phases, under_launcher
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if under_launcher():
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}")
    elif args.gpus > 1 or args.launch or args.dry_run:
        # parent: count devices without any HIP call (AMD SMI / the KFD topology, dist.count_gpus)
        # and start one child per GPU; this process never initialises the GPU and never execs
        if not args.dry_run:
            from mj_envs_amd.dist import count_gpus
            try:
                have = count_gpus()
            except RuntimeError as e:
                raise SystemExit(f"bench.py --gpus {args.gpus}: cannot count GPUs ({e}); refusing to run")
            if have < args.gpus:
                raise SystemExit(f"bench.py --gpus {args.gpus}: only {have} GPU(s) visible; refusing to run "
                                 f"on fewer ranks")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], os.path.abspath(__file__)))

    if args.depth and args.envs_per_gpu == 65536:
        args.envs_per_gpu = 8192
    if args.total_envs:
        w = int(os.environ.get("WORLD_SIZE", "1"))
        if args.total_envs % w:
            raise SystemExit("--total-envs must divide evenly over the ranks")
        args.envs_per_gpu = args.total_envs // w
    shard = shard_from_env(args.envs_per_gpu)
    if args.dry_run:
        return dry_run(args, shard)

    import numpy as np
    import torch
    import torch.distributed as dist
    from mj_envs_amd import _native, perfmodel
    from mj_envs_amd.tasks import attach_task, load_model

    world, rank, local = shard.world, shard.rank, shard.local_rank
    if local >= torch.cuda.device_count():
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s) visible")
    torch.cuda.set_device(local)
    if under_launcher():       # every launched rank, world 1 included, exchanges through RCCL
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    env_id = args.env
    m = attach_task(load_model(env_id), env_id)
    blob = m.to_blob()
    n = args.envs_per_gpu
    sim = _native.Sim(blob, n, device=local, env_offset=shard.env_offset)   # streams keyed by global id
    obs = sim.empty(n, sim.obs_dim)
    act = sim.empty(n, sim.nu)
    rew = sim.empty(n)
    done = sim.empty(n, dtype=torch.uint8)
    goal = sim.empty(n, dtype=torch.uint8)
    sticky = sim.empty(n, dtype=torch.int32)
    totals = EpisodeTotals(n, world, dev)
    tot_ep, tot_ret, tot_suc = totals.rows()          # the kernel writes the send block in place
    sim.reset(obs, seed=SEED_RESET)
    sim.set_episode(ep_len=torch.from_numpy(stagger_phases(n, shard.env_offset, sim.horizon)).to(dev))
    pol = None
    if args.policy == "random-mlp":
        from mj_envs_amd.policy import GaussianMLP
        pol = GaussianMLP(sim.obs_dim, sim.nu, (32, 32), init_log_std=-1.0, seed=0, device=local)
    elif args.policy == "dapg":
        from mj_envs_amd.policy import GaussianMLP
        pol = GaussianMLP.from_npz(os.path.join(REPO, "tests", "golden", f"dapg_{env_id.split('-')[0]}.npz"),
                                   device=local)
    depth = cam = None
    if args.depth:
        from mj_envs_amd.render import free_camera
        cam = free_camera(m, env_id, 64, 64)
        depth = sim.empty(n, 64, 64)

    def gather():
        sim.episode_totals(tot_ep, tot_ret, tot_suc)
        return totals()          # one RCCL all-gather of the packed [3, E] block when launched

    def one_step(k, ev=None):
        if pol is not None:
            pol.act(obs, out=act, sample=args.policy == "random-mlp", seed=SEED_ACT, step=k,
                    env_offset=shard.env_offset)
        else:
            sim.random_actions(act, SEED_ACT, k)
        if ev is not None:
            ev[0].record()
        sim.step(act, obs, rew, done, goal, autoreset=True, seed=SEED_RESET)
        if ev is not None:
            ev[1].record()
        if depth is not None:
            if ev is not None:
                ev[2].record()
            sim.render_depth(depth, cam)
            if ev is not None:
                ev[3].record()
        if (k + 1) % sim.horizon == 0:
            gather()

    preroll = default_preroll(sim.horizon, args.warmup, args.steps) if args.preroll < 0 else args.preroll
    exch_steps = [k for k in range(preroll + args.warmup, preroll + args.warmup + args.steps)
                  if (k + 1) % sim.horizon == 0]
    for k in range(preroll + args.warmup):
        one_step(k)
    e0, r0, s0 = (x.clone() for x in gather())
    sim.clear_status()
    torch.cuda.synchronize()
    pg = dist.is_initialized()
    if pg:
        dist.barrier()
    events = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(preroll + args.warmup + k, events[k])
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern = [e[0].elapsed_time(e[1]) for e in events]
    kern_ms = sum(kern) / args.steps
    depth_ms = sum(e[2].elapsed_time(e[3]) for e in events) / args.steps if depth is not None else None
    e1, r1, s1 = gather()
    # the exchange's own check: the gathered global totals equal the sum of every rank's block
    rank_sums = torch.stack([tot_ep.long().sum(), tot_suc.long().sum()])
    if pg:
        dist.all_reduce(rank_sums, op=dist.ReduceOp.SUM)
    exchange = dict(backend=dist.get_backend() if pg else "local copy", world=world, collective="all_gather_into_tensor"
                    if pg else None, calls=totals.calls, bytes_per_rank_per_call=totals.bytes_per_rank,
                    every_steps=sim.horizon, calls_in_timed_window=len(exch_steps),
                    timed_window_steps=[preroll + args.warmup, preroll + args.warmup + args.steps - 1],
                    exchange_steps_in_window=exch_steps, global_episodes=int(e1.long().sum()),
                    global_successes=int(s1.long().sum()),
                    gathered_equals_rank_sums=bool(int(e1.long().sum()) == int(rank_sums[0])
                                                   and int(s1.long().sum()) == int(rank_sums[1])))
    sim.status(sticky=sticky)
    n_over = int(((sticky & _native.ST_OVERFLOW) != 0).sum())
    n_nan = int(((sticky & (_native.ST_BADQPOS | _native.ST_BADQVEL | _native.ST_BADQACC)) != 0).sum())
    n_wide = int(((sticky & _native.ST_WIDE) != 0).sum())
    t = torch.tensor([elapsed, kern_ms, n_over, n_nan, n_wide], dtype=torch.float64, device=dev)
    if pg:
        dist.all_reduce(t[:2], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[2:], op=dist.ReduceOp.SUM)
    elapsed, kern_ms, n_over, n_nan, n_wide = float(t[0]), float(t[1]), int(t[2]), int(t[3]), int(t[4])
    finite = bool(torch.isfinite(obs).all())

    if rank == 0:
        total_steps = world * n * args.steps
        value = total_steps / elapsed
        flops, counts = perfmodel.step_flops(env_id, m, sim.frame_skip, policy=args.policy)
        flops_dense, _ = perfmodel.step_flops(env_id, m, sim.frame_skip, dense_m=True, policy=args.policy)
        achieved = flops * n / (kern_ms * 1e-3) / 1e12
        bytes_step = perfmodel.step_bytes(sim.nq, sim.nv, sim.nu, sim.obs_dim, sim.nparam)
        build_id = _native.kernel_build_id()
        traffic_raw, traffic_cal, pmc_src, pmc_cal = pmc_traffic(n, env_id, args.policy, build_id)
        # the roofline's traffic: counter bytes divided by the same box's calibration for k_step's
        # access pattern when the summary has one, else the raw counters
        traffic = traffic_cal or traffic_raw
        roof = dict(bound="valu", achieved=round(achieved, 3), peak=perfmodel.PEAK_FP32_TFLOPS,
                    unit="TFLOP/s", frac=round(achieved / perfmodel.PEAK_FP32_TFLOPS, 5), traffic=traffic,
                    kernel=f"k_step<{sim.task_kind}>", nv=sim.nv, kernel_ms=round(kern_ms, 4),
                    kernel_ms_min_max=[round(min(kern), 4), round(max(kern), 4)],
                    flops_per_env_step=round(flops), bytes_per_env_step=bytes_step,
                    work_counts=dict(source=counts["source"], policy=counts["policy"], avg=counts["avg"]),
                    flops_formula="MuJoCo 2.1's algorithms: tree-sparse mj_factorM / mj_solveM for M, dense "
                                  "Cholesky only for the Newton Hessian (perfmodel.py)",
                    r03_dense_formula=dict(flops_per_env_step=round(flops_dense),
                                           frac=round(flops_dense * n / (kern_ms * 1e-3) / 1e12
                                                      / perfmodel.PEAK_FP32_TFLOPS, 5)),
                    hbm_algorithmic_GBps=round(bytes_step * n / (kern_ms * 1e-3) / 1e9, 2),
                    hbm_measured_GBps=round(traffic / (kern_ms * 1e-3) / 1e9, 2) if traffic else None,
                    hbm_measured_frac=round(traffic / (kern_ms * 1e-3) / 1e9 / perfmodel.PEAK_HBM_GBPS, 6)
                    if traffic else None, pmc_source=pmc_src, pmc_calibration=pmc_cal, kernel_build_id=build_id,
                    traffic_bytes_per_env_step=round(traffic / n, 1) if traffic else None,
                    traffic_over_algorithmic=round(traffic / n / bytes_step, 3) if traffic else None,
                    traffic_calibrated=traffic_cal is not None,
                    traffic_raw_bytes_per_env_step=round(traffic_raw / n, 1) if traffic_raw else None,
                    traffic_raw_over_algorithmic=round(traffic_raw / n / bytes_step, 3) if traffic_raw else None,
                    note="FP32 roofline (157.3 TFLOP/s: the vector peak, equal to the fp32 MFMA peak the contact Hessian J'DJ, "
                         "the CRB mass-matrix product and the noslip pair coupling run on); FLOPs "
                         "from perfmodel.py on the oracle's work counts of this regime (work_counts). The HBM figures are far from "
                         "8 TB/s by construction: ~1.1 KB compulsory traffic per env-step (SURVEY 8d), the "
                         "north-star's 40 % of HBM roofline is unreachable on algorithmic bytes")
        workload = (f"{env_id}, {n} envs per GPU (north-star config), random policy, staggered episode phases "
                    f"(+{preroll}-step untimed pre-roll): auto-reset of ~{n // sim.horizon} envs per step inside "
                    f"the timed region; per-env episode totals all-gathered every {sim.horizon} steps")
        if pol is not None:
            workload = workload.replace("random policy", "closed loop with the on-device Gaussian MLP policy "
                                        + ("(mjrl MLP 32x32, random init, sampled actions)"
                                           if args.policy == "random-mlp" else
                                           "(the reference's pretrained DAPG policy, mean actions)"))
        if depth is not None:
            workload = workload.replace("random policy", "random policy + 64x64 depth-camera obs (HIP ray "
                                        "caster, BASELINE config 5)")
            roof["depth_kernel_ms"] = round(depth_ms, 4)
        workload += ", MPR (cylinder) collider in fp64 on fp64 geometry"
        metric = "env-steps/sec at N parallel envs, hammer-v0, 1/2/4/8 MI355X"
        if env_id != "hammer-v0":   # BASELINE config 3 lines are labelled with their own task
            metric = f"env-steps/sec at N parallel envs, {env_id}, 1/2/4/8 MI355X"
        de = e1.long() - e0.long()
        ne = int(de.sum())
        episodes = dict(finished_in_timed_window=ne,
                        mean_return=round(float((r1 - r0).double().sum()) / max(ne, 1), 3),
                        success_pct=round(100.0 * int((s1 - s0).sum()) / max(ne, 1), 3))
        line = dict(metric=metric,
                    value=round(value, 1), unit="env-steps/s", n_gpus=world, steps=args.steps,
                    warmup=args.warmup, ms_per_step=round(elapsed / args.steps * 1e3, 4),
                    higher_is_better=True, scaling="strong" if args.total_envs else "weak", vs_baseline=None,
                    dtype="f32",
                    data="synthetic (Philox U(-1,1) actions, reference reset distribution)",
                    config=dict(workload=workload, envs_per_gpu=n, total_envs=world * n,
                                frame_skip=sim.frame_skip, parallelism=f"env-shard x{world}", preroll=preroll,
                                env_id=env_id, policy=args.policy),
                    roofline=roof, finite=finite, overflow_envs=n_over, bad_state_envs=n_nan,
                    wide_tier_envs=n_wide,
                    capacities=dict(maxcon=sim.maxcon, maxefc=sim.maxefc, maxdense=sim.maxdense,
                                    fast_tier=dict(maxcon=sim.fast_maxcon, maxefc=sim.fast_maxefc,
                                                   maxdense=sim.fast_maxdense),
                                    wide_tier_grid=sim.wide_grid,
                                    note="overflow_envs: envs that dropped a constraint at MuJoCo's own caps "
                                         "(nconmax / njmax, DAPG_assets.xml:4); wide_tier_envs: envs with >= 1 "
                                         "env-step past the fast tier's capacities, re-run in the wide tier"),
                    episodes=episodes, exchange=exchange)
        if world == 1 and not args.no_parity:
            try:
                line["parity_one_step"] = same_run_parity(blob, sim, model=m, pol=pol, obs_now=obs)
                line["parity_one_step"]["actions"] = ("the policy's mean action on the current obs" if pol is not None
                                                      else "Philox U(-1, 1)")
            except Exception as e:
                line["parity_one_step"] = dict(error=str(e))
        if world == 1 and env_id == ENV_ID and depth is None and pol is None and n == 65536 \
                and not args.no_config2:
            line["config2_4096_envs"] = config2(blob, env_id, local)
        if world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(blob, env_id, local)
            except Exception as e:  # the baseline must not hide the GPU number
                line["cpu_baseline"] = dict(value=None, error=str(e))
        print(json.dumps(line), flush=True)
    if pg:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
