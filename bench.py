#!/usr/bin/env python3
"""Benchmark of the MI355X gravity + profile hot path (BASELINE.json configs 2-5).

    python bench.py [--gpus N] [--steps K] [--warmup W]

One step = one full direct-sum force + potential solve of a synthetic
Plummer sphere whose positions / masses are already resident in HBM:
pack this rank's particles into 32-byte source records, all-gather the
records of every rank over RCCL (N > 1), run the fused FP64 direct-sum
kernel for this rank's targets against all sources.

Workload: N_GPU x 1,000,000 particles (1M at N=1 = config 2; 8M at N=8 =
config 4), targets sharded across ranks, every rank sees all sources.
Per-GPU target count is fixed ("weak" in particles); the pair count per
GPU grows with N, which is why the metric is the whole-job pair rate.

Printed (rank 0, one JSON line): metric/value in pairs/s, the roofline of
the direct-sum kernel against the FP64 vector peak (achieved from HIP
events on the library stream), and the CPU baseline (oracle restatement
of direct.rs timed on a bounded target sample on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "pynbody-extras_amd"))
sys.path.insert(0, str(ROOT))

from pynbodyext import _native as nat  # noqa: E402
from pynbodyext.synthetic import plummer  # noqa: E402

FLOP_PER_PAIR = 22            # SURVEY.md §8d, fused force + potential
FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X FP64 vector, AMD spec
N_PER_GPU = 1_000_000
SEEDS = {1_000_000: 1002, 4_000_000: 1003, 8_000_000: 1004}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n-per-gpu", type=int, default=N_PER_GPU)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target duration of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true",
                    help="skip the radial-profile leg (config 3)")
    ap.add_argument("--profile-sizes", default="1000000,16000000,64000000,256000000",
                    help="comma-separated particle counts of the profile size sweep")
    ap.add_argument("--no-tree", action="store_true", help="skip the Barnes-Hut leg (config 5)")
    ap.add_argument("--no-api", action="store_true",
                    help="skip the API-level (host arrays, H2D/D2H inclusive) direct-sum timing")
    ap.add_argument("--tree-n", type=int, default=4_000_000)
    return ap.parse_args()


class Dist:
    """Control plane for one process per GPU, launched by torch.distributed.run.

    Only the environment of the launcher is used (RANK / WORLD_SIZE /
    LOCAL_RANK / MASTER_*); torch is never imported in the worker.  The RCCL
    unique id travels through a node-local rendezvous file, and barrier /
    max-over-ranks run on the RCCL communicator itself, which is also the
    data path (source all-gather).
    """

    def __init__(self):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        # PBX_BENCH_FORCE_DIST=1 runs the multi-rank code path (rendezvous +
        # RCCL communicator) even at world size 1, as a rehearsal.
        self.active = self.world > 1 or os.environ.get("PBX_BENCH_FORCE_DIST") == "1"
        self.comm = None
        if self.active:
            from pynbodyext.parallel import Communicator, FileRendezvous

            rdzv = FileRendezvous(self.rank, self.world)
            uid = rdzv.broadcast(Communicator.unique_id() if self.rank == 0 else None)
            self.comm = Communicator(self.world, self.rank, uid)
            rdzv.cleanup()

    def barrier(self):
        if self.comm is not None:
            self.comm.barrier()

    def max(self, x: float) -> float:
        return self.comm.max(x) if self.comm is not None else x

    def close(self):
        if self.comm is not None:
            self.comm.destroy()
            self.comm = None


def host_cores() -> int:
    """Threads for the multi-core CPU baseline: every core this process may
    use (sched_getaffinity), capped by the box's CPU share when the launcher
    states it in OMP_NUM_THREADS (16 per GPU on the gpurun boxes, where the
    affinity mask shows the whole machine)."""
    cores = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        cores = min(cores, int(omp))
    return max(1, cores)


def cpu_baseline(pos, mass, seconds: float, cores: int | None = None):
    """Oracle restatement of direct.rs (per-target loop, :160-182 / :293-310)
    on a bounded random target sample; returns pairs/s on the host cores."""
    from oracle import gravity as og

    cores = host_cores() if cores is None else int(cores)
    og.set_num_threads(cores)
    n = len(pos)
    rng = np.random.default_rng(0)
    og.direct_subset(pos, mass, np.arange(cores))       # spin up the thread pool
    probe = rng.choice(n, size=4 * cores, replace=False)
    t0 = time.perf_counter()
    og.direct_subset(pos, mass, probe)
    dt = time.perf_counter() - t0
    per_target = dt / len(probe)
    k = int(min(n, max(len(probe), seconds / max(per_target, 1e-9))))
    k = max(cores, (k // cores) * cores)
    # batches of fresh random targets until the sample reaches `seconds`
    # (the probe's per-target estimate is pessimistic: cold caches)
    done, dt = 0, 0.0
    while dt < seconds and done < n:
        kk = min(k, n - done)
        idx = rng.choice(n, size=kk, replace=False)
        t0 = time.perf_counter()
        og.direct_subset(pos, mass, idx)
        dt += time.perf_counter() - t0
        done += kk
    k = done
    return {
        "value": k * (n - 1) / dt,
        "unit": "pairs/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{k} random targets x {n} sources, oracle/gravity_ref.c, {cores} OpenMP "
                  f"threads, {dt:.1f} s",
        **cpu_host(),
    }


def cpu_rows(many: dict, one: dict) -> dict:
    """The CPU baseline rows of a gravity leg: `many` (the box's CPU share,
    host_cores() threads) carries the line; the single-core run and the
    all-affinity-cores figure sit beside it.  The reference's threads=0 is
    rayon's global pool = every core of the machine
    (crates/pynbodyext-rust/src/gravity.rs:87-101); the GPU boxes show 256
    affinity cores but give one GPU's job a share of 16 (OMP_NUM_THREADS,
    the harness's rule for worker pools), so the all-cores row is the
    16-thread rate scaled linearly to the affinity count — an upper bound
    on what rayon could reach there (perfect scaling), not a run."""
    aff = len(os.sched_getaffinity(0))
    many["single_core_value"] = one["value"]
    many["threads_scaling_efficiency"] = many["value"] / (many["cores"] * one["value"])
    many["all_affinity_cores_bound_value"] = many["value"] * aff / many["cores"]
    many["single_core"] = {k: one[k] for k in ("value", "cores", "sample")}
    many["all_affinity_cores_bound"] = {
        "value": many["value"] * aff / many["cores"], "cores": aff,
        "kind": "linear extrapolation (upper bound), not run",
        "note": f"{many['cores']}-thread rate x {aff}/{many['cores']}: the reference's rayon "
                "pool on every affinity core with perfect scaling; not run because a one-GPU "
                "job's CPU share on the box is OMP_NUM_THREADS threads"}
    return many


PROFILE_BYTES_PER_PARTICLE = 49  # equaln profile, algorithmic HBM bytes / input particle
HBM_PEAK_GBS = 8000.0


def profile_parity(dev, res, ref) -> dict:
    """The last timed step's results against oracle/profile_ref.radial_profile
    on the same particles (outside the timed region): edges, counts and the
    CSR (binind, bins.py:383-393) bit-exact; Σm and mass-weighted <r> per bin
    (proarray.py:320-328) relative to the oracle's numpy sums."""
    edges, msum, rmom = res
    perm, offs = dev.csr()
    with np.errstate(invalid="ignore", divide="ignore"):
        rmean = rmom[:, 1] / rmom[:, 0]  # weighted Mean: Σ(r·m) / Σm
        ms = np.abs(msum - ref["mass_sum"]) / np.abs(ref["mass_sum"])
        rm = np.abs(rmean - ref["r_mean"]) / np.abs(ref["r_mean"])
    return {
        "edges_bit_exact": bool(np.array_equal(edges, ref["edges"])),
        "counts_bit_exact": bool(np.array_equal(dev.counts, ref["counts"])),
        "csr_bit_exact": bool(np.array_equal(offs, ref["offsets"]) and np.array_equal(perm, ref["perm"])),
        "mass_sum_max_rel": float(np.nanmax(ms)),
        "r_mean_max_rel": float(np.nanmax(rm)),
        "n_kept": int(len(ref["x"])),
    }


def dist_profile_parity(rank: int, world: int, n: int, res, counts):
    """Rank 0: the global profile (edges, counts, Σm) against the oracle on
    the concatenation of every rank's particles (regenerated from the seeds,
    rank order), outside the timed region; other ranks return None."""
    if rank != 0:
        return None
    from oracle import profile_ref as pr
    from pynbodyext.synthetic import family_slices

    dm = family_slices(n)["dm"]
    rs, ms = [], []
    for r in range(world):
        pos, mass = plummer(n, seed=SEEDS.get(n, 1002) + 7919 * r)
        keep = pr.sphere_mask(pos, 10.0)
        keep[dm.stop:] = False
        rs.append(pr.radial_r(pos[keep]))
        ms.append(mass[keep])
    x, w = np.concatenate(rs), np.concatenate(ms)
    edges = pr.edges_equaln(x, 128)
    perm, offs, cnt = pr.assign(x, edges)
    msum, _ = pr.compute(w, w, perm, offs, "sum")
    e, s, _ = res
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.abs(s - msum) / np.abs(msum)
    return {"ranks": world, "n_kept_all": int(len(x)),
            "edges_bit_exact": bool(np.array_equal(e, edges)),
            "counts_bit_exact": bool(np.array_equal(counts, cnt)),
            "mass_sum_max_rel": float(np.nanmax(rel))}


N_CHANGING = 4  # distinct snapshots one handle cycles through (the base one + 3)


def _stats_delta(a: dict, b: dict) -> dict:
    return {k: b[k] - a[k] for k in a}


def changing_snapshots(n: int, steps: int, single, dev, d_pos, d_mass, e0, e1, cpu: bool) -> dict:
    """The profile step on inputs that change between calls: one handle
    cycles through N_CHANGING distinct snapshots of the same workload (the
    base snapshot and 3 more Plummer spheres of other seeds, drawn by
    synthetic.plummer_chunked), every call a different particle set than the
    previous one, as a user profiling successive outputs of a simulation
    would.  The reference recomputes the bins on every BinsSet.__call__
    (bins.py:397-457).  Reports the median stream / wall time per call and
    the hit rates of the handle's speculation; the last snapshot's results
    are checked bit-exact against a fresh handle's first call on it (and, at
    n <= 16M with the CPU legs on, against the oracle)."""
    from pynbodyext.profiles._device import DeviceBins
    from pynbodyext.synthetic import family_slices, plummer_chunked

    snaps = [(d_pos, d_mass, None)]
    for k in range(1, N_CHANGING):
        p, m = plummer_chunked(n, seed=SEEDS.get(n, 1002) + 104729 * k,
                               threads=min(16, host_cores()))
        snaps.append((nat.DeviceArray.from_host(p), nat.DeviceArray.from_host(m),
                      p if (cpu and n <= 16_000_000) else None))
        del m
    calls = max(8 * N_CHANGING, steps)
    calls -= calls % N_CHANGING
    s0 = (dev.spec_stats(), dev.level0_stats(), dev.mono_stats(), dev.path_stats())
    for k in range(N_CHANGING):  # every snapshot once before the timed calls
        single(snaps[k][0].ptr, snaps[k][1].ptr, dev)
    nat.synchronize()
    s1 = (dev.spec_stats(), dev.level0_stats(), dev.mono_stats(), dev.path_stats())
    # per call (an event pair and a sync around each: the distribution), then
    # the same calls back to back between one event pair and one sync — the
    # bench's step bracket; the per-call events and sync add ~15 us of
    # measurement to every call, which the credited (batch) figure leaves out
    ct, cd = [], []
    res = None
    for i in range(calls):
        pp, mp, _ = snaps[i % N_CHANGING]
        t0 = time.perf_counter()
        e0.record()
        res = single(pp.ptr, mp.ptr, dev)
        e1.record()
        nat.synchronize()
        ct.append(time.perf_counter() - t0)
        cd.append(e0.elapsed_ms(e1))
    nat.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for i in range(calls):
        pp, mp, _ = snaps[i % N_CHANGING]
        res = single(pp.ptr, mp.ptr, dev)
    e1.record()
    nat.synchronize()
    bt = (time.perf_counter() - t0) / calls
    bd = e0.elapsed_ms(e1) / calls
    s2 = (dev.spec_stats(), dev.level0_stats(), dev.mono_stats(), dev.path_stats())
    last = snaps[(calls - 1) % N_CHANGING]
    fresh = DeviceBins()
    fr = single(last[0].ptr, last[1].ptr, fresh)
    perm_a, offs_a = dev.csr()
    perm_b, offs_b = fresh.csr()
    with np.errstate(invalid="ignore", divide="ignore"):
        ms = np.abs(res[1] - fr[1]) / np.abs(fr[1])
    check = {"vs": "a fresh handle's first call on the same snapshot (no speculation)",
             "edges_bit_exact": bool(np.array_equal(res[0], fr[0])),
             "counts_bit_exact": bool(np.array_equal(dev.counts, fresh.counts)),
             "csr_bit_exact": bool(np.array_equal(perm_a, perm_b) and np.array_equal(offs_a, offs_b)),
             "mass_sum_max_rel": float(np.nanmax(ms))}
    if last[2] is not None:
        from oracle import profile_ref as pr

        dm = family_slices(n)["dm"]
        mask = pr.sphere_mask(last[2], 10.0)
        mask[dm.stop:] = False
        ref = pr.radial_profile(last[2], np.full(n, 1.0 / n), mask, "equaln", 128)
        check["vs_oracle"] = profile_parity(dev, res, ref)
    fresh.close()
    for pp, mp, _ in snaps[1:]:
        pp.free()
        mp.free()
    td = bd
    delta = [dict(zip(("speculation", "level0", "one_launch", "path"),
                      [_stats_delta(a, b) for a, b in zip(x, y)])) for x, y in ((s0, s1), (s1, s2))]
    return {"snapshots": N_CHANGING, "calls": calls, "stream_ms": td,
            "ms": bt * 1e3,
            "timing": "stream_ms / ms: `calls` back-to-back calls between one event pair and one "
                      "sync, per call; per_call: an event pair and a sync around every call "
                      "(median, p90)",
            "per_call": {"stream_ms": float(np.median(cd)),
                         "stream_ms_p90": float(np.percentile(cd, 90)),
                         "ms": float(np.median(ct)) * 1e3},
            "particles_per_s_stream": n / (td * 1e-3),
            "particles_per_s_wall": n / bt,
            "hbm_gbs_algorithmic": n * PROFILE_BYTES_PER_PARTICLE / (td * 1e-3) / 1e9,
            "frac": n * PROFILE_BYTES_PER_PARTICLE / (td * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "handle_stats_timed_calls": delta[1], "handle_stats_first_pass": delta[0],
            "parity": check,
            "seeds": [SEEDS.get(n, 1002)] + [SEEDS.get(n, 1002) + 104729 * k
                                             for k in range(1, N_CHANGING)]}


def bench_profile(sizes, steps: int, warmup: int, cpu: bool, dist=None):
    """Config 3: RadialProfileBuilder(ndim=3, weight='mass', equaln, 128 bins)
    behind Sphere(R=10) & FamilyFilter('dm'), positions / masses resident in
    HBM.  One step = fused select (mask + r + compaction) -> equaln edges ->
    bin assignment + counts -> CSR (binind) built in HBM -> per-bin Σ mass and
    mass-weighted <r>.  particles/s counts every INPUT particle.

    With several ranks (weak scaling): every rank holds n particles of its own
    (seed + 7919 rank), the edges are the global equaln, counts and sums are
    global (ShardedProfile.radial_equaln: the same kernels with RCCL
    all-reduces of the key range, the level-0 digit histogram, the gathered
    group keys and the packed results between them; PBX_BENCH_STAGED=1: the
    staged host-driven distributed radix select instead);
    particles/s = world * n / (max-over-ranks step time).  Rank 0 checks the
    first size against the oracle on all ranks' particles."""
    from pynbodyext.parallel import ShardedProfile
    from pynbodyext.profiles._device import SRC_NONE, SRC_W, SRC_X, DeviceBins
    from pynbodyext.synthetic import family_slices

    comm = dist.comm if dist is not None else None
    world = dist.world if dist is not None else 1
    rank = dist.rank if dist is not None else 0
    out = []
    for n in sizes:
        pos, mass = plummer(n, seed=SEEDS.get(n, 1002) + 7919 * rank)
        dm = family_slices(n)["dm"]
        d_pos = nat.DeviceArray.from_host(pos)
        d_mass = nat.DeviceArray.from_host(mass)
        dev = DeviceBins()
        # the positions / masses stay resident and unchanged for the whole
        # leg: a repeated call may speculate and keep no copy of x
        # (pbx_profile_set_source_stable)
        dev.set_source_stable(True)
        sp = ShardedProfile(comm, dev, offset=rank * n)
        e0, e1 = nat.Event(), nat.Event()

        # the columns these two statistics read (proarray Sum: Σf; weighted
        # Mean: Σw, Σf·w) — what pynbodyext.profiles requests for them
        stats = [(SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, (1 << 0) | (1 << 1))]

        staged = os.environ.get("PBX_BENCH_STAGED") == "1"

        def single(pp, mp, into):  # selection, edges, counts, CSR and sums: one host round trip
            _, edges, _, (msum, rmean) = DeviceBins.radial_equaln(
                pp, mp, nbins=128, sphere=((0.0, 0.0, 0.0), 10.0),
                families=[(dm.start, dm.stop)], ndim=3, stats=stats, csr=True,
                on_device=True, n=n, into=into)
            return edges, msum[:, 3], rmean

        def step():
            if comm is None:
                return single(d_pos.ptr, d_mass.ptr, dev)
            if not staged:  # the same pipeline with device all-reduces between its kernels
                edges, counts, (msum, rmean) = sp.radial_equaln(
                    d_pos.ptr, d_mass.ptr, nbins=128, sphere=((0.0, 0.0, 0.0), 10.0),
                    families=[(dm.start, dm.stop)], ndim=3, stats=stats, csr=True,
                    on_device=True, n=n)
                step.counts = counts
                return edges, msum[:, 3], rmean
            DeviceBins.select(d_pos.ptr, d_mass.ptr, sphere=((0.0, 0.0, 0.0), 10.0),
                              families=[(dm.start, dm.stop)], ndim=3, on_device=True, n=n, into=dev)
            edges = sp.edges_equaln(128)
            step.counts = sp.assign(edges)
            dev.build_csr_on_device()
            msum = sp.moments(*stats[0])[:, 3]
            rmean = sp.moments(*stats[1])
            return edges, msum, rmean

        for _ in range(warmup):
            step()
        nat.synchronize()
        times, dev_ms = [], []
        for _ in range(steps):
            if dist is not None:
                dist.barrier()
            t0 = time.perf_counter()
            e0.record()
            res = step()
            e1.record()
            nat.synchronize()
            dt = time.perf_counter() - t0
            times.append(dist.max(dt) if dist is not None else dt)
            dev_ms.append(e0.elapsed_ms(e1))
        t = float(np.median(times))
        td = float(np.median(dev_ms)) * 1e-3
        per_call = {"stream_ms": td * 1e3, "ms": t * 1e3}
        if dist is not None:
            td = dist.max(td)
        else:  # the same steps back to back in one bracket (see changing_snapshots)
            nat.synchronize()
            t0 = time.perf_counter()
            e0.record()
            for _ in range(steps):
                res = step()
            e1.record()
            nat.synchronize()
            t = (time.perf_counter() - t0) / steps
            td = e0.elapsed_ms(e1) * 1e-3 / steps
        n_all = n * world
        row = {"n": n_all, "n_per_gpu": n, "n_kept_rank0": dev.n, "ms": t * 1e3,
               "particles_per_s": n_all / t,
               "hbm_gbs_algorithmic": n_all * PROFILE_BYTES_PER_PARTICLE / td / 1e9,
               "hbm_gbs_algorithmic_per_gpu": n * PROFILE_BYTES_PER_PARTICLE / td / 1e9,
               "stream_ms": td * 1e3}
        if dist is None:
            # the rows above are ONE snapshot called again and again (a profile
            # per statistic): the handle reuses the previous call's level-0
            # geometry and speculates on its bin table and edges
            row["identical_snapshot"] = {"stream_ms": row["stream_ms"], "ms": row["ms"],
                                         "per_call": per_call,
                                         "path": dev.path_stats(), "mono": dev.mono_stats(),
                                         "level0_hinted_calls": dev.level0_stats(),
                                         "speculated_calls": dev.spec_stats()}
            # a first call on every step: no earlier geometry or speculation state
            ct, cd = [], []
            nc = max(20, steps // 10)
            for _ in range(nc):
                dev.forget_history()  # the next call runs as the handle's first
                t0 = time.perf_counter()
                e0.record()
                step()
                e1.record()
                nat.synchronize()
                ct.append(time.perf_counter() - t0)
                cd.append(e0.elapsed_ms(e1))
            nat.synchronize()
            t0 = time.perf_counter()
            e0.record()
            for _ in range(nc):
                dev.forget_history()
                step()
            e1.record()
            nat.synchronize()
            row["cold_ms"] = (time.perf_counter() - t0) / nc * 1e3
            row["cold_stream_ms"] = e0.elapsed_ms(e1) / nc
            row["cold_per_call"] = {"stream_ms": float(np.median(cd)),
                                    "ms": float(np.median(ct)) * 1e3}
            row["cold_note"] = ("every call a handle's first (forget_history: no earlier "
                                "geometry or speculation state)")
            row["changing"] = changing_snapshots(n, steps, single, dev, d_pos, d_mass, e0, e1,
                                                 cpu)
            # the handle's CSR of the base snapshot again (the parity check below)
            res = single(d_pos.ptr, d_mass.ptr, dev)
        out.append(row)
        if cpu and world == 1:
            from oracle import profile_ref as pr

            mask = pr.sphere_mask(pos, 10.0)
            mask[dm.stop:] = False
            if n == sizes[0]:
                # the full workload, repeated until ~10 s of CPU time
                reps, tc = 0, 0.0
                while tc < 10.0 and reps < 1000:
                    t0 = time.perf_counter()
                    ref = pr.radial_profile(pos, mass, mask, "equaln", 128)
                    tc += time.perf_counter() - t0
                    reps += 1
                row["cpu_baseline"] = {
                    "value": reps * n / tc, "unit": "particles/s", "cores": 1, "kind": "port",
                    "sample": f"full {n}-particle workload x {reps}, oracle/profile_ref.py (numpy "
                              f"restatement of bins.py/proarray.py), 1 thread, {tc:.1f} s",
                    **cpu_host()}
            else:
                ref = pr.radial_profile(pos, mass, mask, "equaln", 128)
            row["parity_vs_oracle"] = profile_parity(dev, res, ref)
        if dist is not None and n == sizes[0] and world > 1:
            row["parity_vs_oracle"] = dist_profile_parity(rank, world, n, res, step.counts)
        dev.close()
        d_pos.free()
        d_mass.free()
    return out


TREE_FLOP_NODE = 94   # order-3 force+potential node interaction incl. opening test (ISA count, FMA = 2)
TREE_FLOP_PP = 22     # leaf pair, same algorithmic count as the direct sum


def tree_outputs(solver, n: int):
    """(potential, acceleration) of the solver's last walk in original
    particle order (the walk writes them in leaf order)."""
    pot = np.empty(n)
    acc = np.empty((n, 3))
    idx = nat.DeviceArray(8 * n)
    solver.tree._leaf_particles_device(0, n, None, None, idx.ptr)
    order = np.empty(n, dtype=np.int64)
    idx.download(order)
    tmp = np.empty(n)
    solver.d_pot.download(tmp)
    pot[order] = tmp
    tmp3 = np.empty((n, 3))
    solver.d_acc.download(tmp3)
    acc[order] = tmp3
    idx.free()
    return pot, acc


def tree_cpu_baseline(pos, mass, seconds: float, theta: float, gpu: dict,
                      cores: int | None = None):
    """Oracle restatement of tree.rs (serial build + payload like the
    reference, OpenMP walk over a bounded random target sample); returns the
    extrapolated full-solve rate in effective pairs/s and, for every
    (potential, acceleration) pair in ``gpu``, the parity of the GPU values on
    the sampled targets."""
    from oracle import gravity as og
    from oracle import tree as ot

    cores = host_cores() if cores is None else int(cores)
    og.set_num_threads(cores)
    n = len(pos)
    rng = np.random.default_rng(0)
    t0 = time.perf_counter()
    ref = ot.RefOctree(pos, mass, 8, 3)
    t_build = time.perf_counter() - t0
    probe = rng.choice(n, size=64 * cores, replace=False)
    t0 = time.perf_counter()
    ref.compute_subset(probe, theta)
    per_target = (time.perf_counter() - t0) / len(probe)
    k = int(min(n, max(len(probe), max(seconds - t_build, 1.0) / max(per_target, 1e-12))))
    idx = rng.choice(n, size=k, replace=False)
    t0 = time.perf_counter()
    pot, acc, _, _ = ref.compute_subset(idx, theta)
    t_walk = time.perf_counter() - t0
    t_full = t_build + t_walk * n / k
    par = {}
    for name, (gpu_pot, gpu_acc) in gpu.items():
        par[name] = {"targets_checked": k,
                     "pot_max_rel": float(np.max(np.abs(gpu_pot[idx] - pot) / np.abs(pot))),
                     "acc_max_rel": float(np.max(np.linalg.norm(gpu_acc[idx] - acc, axis=1) /
                                                 np.linalg.norm(acc, axis=1)))}
    return {
        "value": float(n) * float(n - 1) / t_full,
        "unit": "effective pairs/s",
        "cores": cores,
        "kind": "port",
        "sample": f"oracle/tree_ref.c: serial build+payload of all {n} particles ({t_build:.1f} s) + "
                  f"walk of {k} random targets on {cores} OpenMP threads ({t_walk:.1f} s), "
                  f"full solve extrapolated to {t_full:.1f} s",
        **cpu_host(),
    }, par


def bench_tree(dist, n: int, steps: int, warmup: int, cpu: bool, cpu_seconds: float):
    """Config 5: Barnes-Hut tree (theta=0.5, leaf 8, order 3 = Gravity's
    TreeOptions defaults, base.py:82-100) force + potential of an n-particle
    Plummer sphere resident in HBM, then the 256-bin log radial profile
    (0.01..50) of the mass-weighted potential.  One step = device octree build
    + mass/multipole payload + walk (all particles, self skipped) + profile
    (r, bin assignment, per-bin sums of m and m*phi).  With N ranks (strong
    scaling, n fixed): every rank builds the tree, walks its cost-balanced
    range of the leaf-ordered targets and the profile partials are summed by
    one RCCL all-reduce (pynbodyext.parallel.ShardedTree)."""
    from pynbodyext.parallel import ShardedTree
    from pynbodyext.profiles._device import DeviceBins

    theta = 0.5
    pos, mass = plummer(n, seed=SEEDS.get(n, 1003))
    d_pos = nat.DeviceArray.from_host(pos)
    d_mass = nat.DeviceArray.from_host(mass)
    edges = np.logspace(np.log10(0.01), np.log10(50.0), 257)
    prof = DeviceBins()
    solver = ShardedTree(dist.comm, n, d_pos, d_mass, 8, 3, theta)
    ev = [nat.Event() for _ in range(6)]

    def step():
        # everything a step needs is inside it: build, the cost-balanced
        # ranges (costs carried from the previous step's walk), the walk and
        # its cost all-gather, the profile and its all-reduce
        ev[0].record()
        solver.build()
        ev[1].record()
        solver.balance()
        ev[2].record()
        solver.walk(share=False)
        ev[3].record()
        solver.share_costs()
        ev[4].record()
        mom = solver.profile(prof, edges)
        ev[5].record()
        return mom

    for _ in range(warmup):
        step()
    nat.synchronize()
    dist.barrier()
    if dist.world == 1:
        # the interaction counts of the (one, whole) range were taken by the
        # warm-up walk; the timed walks run without the statistics'
        # instrumentation (pbx_octree_set_walk_counters: same decisions and
        # sums, ~7 fewer scalar operations per wave step)
        solver.set_walk_counters(False)
    wall, parts = [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        mom = step()
        nat.synchronize()
        dist.barrier()
        wall.append(dist.max(time.perf_counter() - t0))
        parts.append([ev[i].elapsed_ms(ev[i + 1]) for i in range(5)])
    t = float(np.median(wall))
    build_ms, bal_ms, walk_ms, share_ms, prof_ms = (float(np.median([p[i] for p in parts]))
                                                    for i in range(5))
    info = solver.info
    check = cpu and dist.world == 1 and dist.rank == 0
    # the outputs of the last timed (fast-mode, headline) step, before the
    # precise-mode steps below overwrite them
    fast_out = tree_outputs(solver, n) if check else None
    solver.set_walk_counters(True)
    with nat.precise_mode(True):  # the walk in precise mode, beside the fast headline
        pw = []
        for _ in range(3):
            step()
            nat.synchronize()
            dist.barrier()
            pw.append(ev[2].elapsed_ms(ev[3]))
        walk_precise_ms = dist.max(float(np.median(pw[1:])))
    first, count = solver.ranges[dist.rank] if solver.ranges else (0, n)
    flops = info["node_interactions"] * TREE_FLOP_NODE + info["leaf_pairs"] * TREE_FLOP_PP
    achieved = flops / (walk_ms * 1e-3) / 1e12
    walk_max = dist.max(walk_ms)
    with np.errstate(invalid="ignore", divide="ignore"):
        phi_profile = mom[:, 1] / mom[:, 0]
    out = {
        "metric": "effective particle-pairs/sec (Barnes-Hut force+potential + 256-bin potential profile)",
        "value": float(n) * float(n - 1) / t,
        "unit": "effective pairs/s",
        "n_gpus": dist.world,
        "scaling": "strong",
        "ms_per_step": t * 1e3,
        "config": {"workload": f"{n}-particle Plummer sphere, octree theta=0.5 leaf 8 multipole "
                               "order 3 (Newtonian), force+potential at every particle, then "
                               "RadialProfile log 256 bins [0.01, 50] of the mass-weighted potential",
                   "n_particles": n, "nodes": info["nodes"], "levels": info["levels"],
                   "parallelism": f"tree replicated, leaf-ordered targets cost-balanced x{dist.world}"
                                  + (", RCCL all-reduce of profile partials" if dist.world > 1 else "")},
        "phases_ms": {"build_and_payload": build_ms, "balance": bal_ms,
                      "walk": walk_ms, "walk_max_over_ranks": walk_max, "cost_share": share_ms,
                      "profile": prof_ms},
        "balance": "timed in every step: ranges from the previous step's per-target interaction "
                   "counts, carried in original particle order (no extra walk)",
        "interactions": {"node": info["node_interactions"], "leaf_pairs": info["leaf_pairs"],
                         "per_target": (info["node_interactions"] + info["leaf_pairs"]) / max(count, 1),
                         "simd_lane_efficiency": info["active_lane_steps"] /
                         max(1, 64 * info["wave_steps"]), "targets_rank0": count},
        "roofline": {"bound": "fp64-valu", "achieved": achieved, "peak": FP64_VECTOR_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / FP64_VECTOR_PEAK_TFLOPS,
                     "traffic": pmc_traffic("tree")[0], "kernel": "walk_kernel<order 3, pot+acc>",
                     "flop_per_node": TREE_FLOP_NODE, "flop_per_leaf_pair": TREE_FLOP_PP,
                     "kernel_ms": walk_ms, "mode": "precise" if nat.get_precise() else "fast",
                     "traffic_source": pmc_traffic("tree")[1],
                     "precise": precise_row(flops, walk_precise_ms)},
        "profile_check": {"bins_nonempty": int(np.sum(mom[:, 0] > 0)),
                          "phi_innermost_bin": float(phi_profile[mom[:, 0] > 0][0]),
                          "phi_outermost_bin": float(phi_profile[mom[:, 0] > 0][-1])},
    }
    if check:
        precise_out = tree_outputs(solver, n)  # the last precise-mode step's
        many, par = tree_cpu_baseline(pos, mass, cpu_seconds, theta,
                                      {"fast": fast_out, "precise": precise_out})
        # the headline (fast-mode) walk's outputs; the precise walk's beside them
        out["parity_vs_oracle"] = {**par["fast"], "mode": "fast (the timed walk)",
                                   "precise_pot_max_rel": par["precise"]["pot_max_rel"],
                                   "precise_acc_max_rel": par["precise"]["acc_max_rel"]}
        one, _ = tree_cpu_baseline(pos, mass, cpu_seconds / 2, theta, {}, cores=1)
        out["cpu_baseline"] = cpu_rows(many, one)
    solver.close()
    prof.close()
    d_pos.free()
    d_mass.free()
    return out


def bench_api(pos, mass, reps: int = 2) -> dict:
    """API-level direct sum (BASELINE.md §3 GPU timing rules: "API time
    includes H2D/D2H"): the reference's host-array entry points
    pynbodyext._rust.direct_potentials_py / direct_accelerations_py
    (gravity.rs:448-512, :585-644) on the same 1M particles — upload,
    kernel, download and host-side checks inside the timed call."""
    from pynbodyext import _rust

    n = len(pos)
    _rust.direct_potentials_py(pos, mass)      # warm: device workspace allocated
    _rust.direct_accelerations_py(pos, mass)
    tp, ta = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        _rust.direct_potentials_py(pos, mass)
        tp.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        _rust.direct_accelerations_py(pos, mass)
        ta.append(time.perf_counter() - t0)
    p, a = float(np.median(tp)), float(np.median(ta))
    pairs = float(n) * float(n - 1)
    return {"n": n, "potentials_ms": p * 1e3, "accelerations_ms": a * 1e3,
            "potentials_pairs_per_s": pairs / p, "accelerations_pairs_per_s": pairs / a,
            "note": "host numpy arrays in and out (PCIe-inclusive), one call per quantity as the "
                    "reference API has; the bench's value is the device-resident fused solve"}


def bench_profile_api(sizes=(1_000_000, 16_000_000), reps: int = 5) -> dict:
    """Config 3 through the API a reference user calls, on HOST arrays
    (PCIe-inclusive; the bench's profile value is the device-resident
    pipeline): RadialProfileBuilder(ndim=3, weight="mass", bins_type="equaln",
    nbins=128).filter(Sphere(10) & FamilyFilter("dm"))(sim) with the two
    statistics read (profiles/base.py:75-140, spatial_profile.py:30-35), and
    the profile drop-in's seams (integration/pynbodyext_mi355x_profiles.py:
    bins.py:720-746 equaln fused with :346-395 assignment + CSR read-back,
    and the Σ mass of proarray.py:272-334) on the host r of the kept
    particles, as the reference's BinsSet calls them."""
    import ctypes
    import importlib.util
    from types import SimpleNamespace

    from pynbodyext.filters import FamilyFilter, Sphere
    from pynbodyext.profiles import RadialProfileBuilder
    from pynbodyext.synthetic import family_slices, plummer_snapshot

    spec = importlib.util.spec_from_file_location(
        "pbx_integration_bench", ROOT / "integration" / "pynbodyext_mi355x_profiles.py")
    integ = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(integ)
    integ._load(str(nat.lib_path()))
    rows = []
    for n in sizes:
        sim = plummer_snapshot(n, seed=SEEDS.get(n, 1002))
        builder = RadialProfileBuilder(ndim=3, weight="mass", bins_type="equaln",
                                       nbins=128).filter(Sphere(10.0) & FamilyFilter("dm"))

        def call():
            prof = builder(sim)
            return prof, np.asarray(prof["mass"]["sum"]), np.asarray(prof["r"])

        call()
        tb = []
        for _ in range(reps):
            t0 = time.perf_counter()
            prof, msum, rmean = call()
            tb.append(time.perf_counter() - t0)
        kept = len(prof.sim)
        # the same call reading the view's r and masses onto the host too (the
        # builder leaves them on the device until read)
        ta = []
        for _ in range(reps):
            t0 = time.perf_counter()
            prof, msum, rmean = call()
            np.asarray(prof.sim["r"]), np.asarray(prof.sim["mass"])
            ta.append(time.perf_counter() - t0)
        # the seams on the host r of the same kept particles
        pos, mass = np.asarray(sim["pos"]), np.asarray(sim["mass"])
        dm = family_slices(n)["dm"]
        p = pos[dm]
        r2 = (p[:, 0] * p[:, 0] + p[:, 1] * p[:, 1]) + p[:, 2] * p[:, 2]
        keep = r2 < 100.0
        x = np.sqrt(r2[keep])
        w = np.asarray(mass[dm])[keep]

        def seams():
            bs = SimpleNamespace(nbins=128, _bin_min=None, _bin_max=None)
            edges = integ._equal_number_bins_algorithm(bs, x)
            binind, counts = integ._assign_particles(bs, x, edges)
            m = bs.__dict__["_pbx_handle"].moments(w, None, 1 << 3)
            bs.__dict__["_pbx_handle"].close()
            return edges, counts, m

        seams()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            edges, counts, m = seams()
            ts.append(time.perf_counter() - t0)
        same = (np.array_equal(edges, np.asarray(prof.bin_edges)) and
                np.array_equal(counts, np.asarray(prof.npart_bins)))
        b, sm, ba = float(np.median(tb)), float(np.median(ts)), float(np.median(ta))
        # the bound: the bytes the selection reads (positions + masses of the
        # family's span) over this box's pinned host -> device rate
        sel_bytes = (dm.stop - dm.start) * (24 + 8)
        pin, stg = ctypes.c_double(), ctypes.c_double()
        nat.call("pbx_measure_h2d", sel_bytes, ctypes.byref(pin), ctypes.byref(stg))
        bound_ms = sel_bytes / (pin.value * 1e9) * 1e3
        rows.append({"n": n, "kept": kept,
                     "builder_ms": b * 1e3, "builder_particles_per_s": n / b,
                     "selection_bytes": sel_bytes, "pinned_h2d_gbs": pin.value,
                     "staged_h2d_gbs": stg.value, "bound_ms": bound_ms,
                     "builder_over_bound": b * 1e3 / bound_ms,
                     "builder_read_all_ms": ba * 1e3,
                     "read_all_over_bound": ba * 1e3 / bound_ms,
                     "seams_ms": sm * 1e3, "seams_kept_per_s": kept / sm,
                     "seams_equal_builder": bool(same)})
        del sim, prof
    return {"rows": rows,
            "note": "host numpy in and out (positions / masses of the family span staged to HBM "
                    "through pinned chunks inside the call for the builder, the view's indices "
                    "read back as int32 widened on the host, r and the kept masses left on the "
                    "device until read — builder_read_all_ms reads both too; r uploaded, the "
                    "int64 CSR read back for the seams): PCIe-inclusive user-facing times, not "
                    "the bench value; bound_ms = selection_bytes / pinned_h2d_gbs "
                    "(pbx_measure_h2d)"}


def pmc_profile_step_bytes(n: int, inputs: str = "identical"):
    """HBM bytes of one n-particle profile call from the committed PMC
    summary (profiles/pmc_profile_<N>M.json, collected at its "n"): a call on
    a changing snapshot ("changing": hbm_bytes_per_step_changing) or a
    repeated one ("identical": hbm_bytes_per_step)."""
    for f in (ROOT / "profiles" / f"pmc_profile_{n // 1_000_000}M.json",
              ROOT / "profiles" / "pmc_profile_latest.json"):
        if not f.exists():
            continue
        try:
            d = json.loads(f.read_text())
            if int(d.get("n", 64_000_000)) == n:
                key = "hbm_bytes_per_step_changing" if inputs == "changing" else "hbm_bytes_per_step"
                return d.get(key), str(f.relative_to(ROOT))
        except Exception:
            continue
    return None, None


def pmc_traffic(which: str = "direct"):
    """HBM bytes per launch of a bench kernel from the committed rocprofv3
    PMC summary (profiles/pmc_<which>_latest.json, tools/pmc_summary.py), or None."""
    f = ROOT / "profiles" / f"pmc_{which}_latest.json"
    if not f.exists():
        return None, None
    try:
        d = json.loads(f.read_text())
        return d.get("hbm_bytes_per_launch"), str(f.relative_to(ROOT))
    except Exception:
        return None, None


def launch_ranks(args) -> int:
    """``--gpus N`` (N > 1) without a launcher: start N rank processes of this
    same command under torch.distributed.run (one process per GPU) BEFORE
    this process touches the GPU, and return their exit status."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, env=env).returncode


def cpu_host() -> dict:
    """Host CPU model and the cores this process may use."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(),
            "affinity_cores": len(os.sched_getaffinity(0))}


# The symmetric kernel evaluates each UNORDERED pair once: 18 FP64 VALU
# instructions + 1 v_rsq_f64 (csrc/direct_sym.hip, fast mode), i.e. half the
# instructions of two ordered pairs.  The FP64 vector pipe issues one wave64
# FP64 instruction per 4 cycles per SIMD: 256 CUs x 4 SIMDs x 16 lanes x
# 2.4 GHz = 39.3e12 lane-instructions/s (78.6 TF counts an FMA as 2).
SYM_INSTR_PER_UNORDERED_PAIR = 19
FP64_LANE_INSTR_PEAK = 256 * 4 * 16 * 2.4e9


def precise_row(flop: float, kernel_ms: float) -> dict:
    """The kernel in precise mode (pbx_set_precise(1): 1/r Newton-refined,
    the reference's arithmetic to rounding) beside the fast-mode headline."""
    tf = flop / (kernel_ms * 1e-3) / 1e12
    return {"kernel_ms": kernel_ms, "achieved": tf, "frac": tf / FP64_VECTOR_PEAK_TFLOPS,
            "mode": "precise", "note": "same launch, pbx_set_precise(1); not the headline"}


def executed_issue(symmetric: bool, pairs_launch: float, kern_ms: float) -> dict:
    if not symmetric:
        return {}
    instr = pairs_launch / 2 * SYM_INSTR_PER_UNORDERED_PAIR
    rate = instr / (kern_ms * 1e-3)
    return {"executed_fp64_instr_per_unordered_pair": SYM_INSTR_PER_UNORDERED_PAIR,
            "executed_issue_frac": rate / FP64_LANE_INSTR_PEAK}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE {world_env}", file=sys.stderr)
        sys.exit(2)
    if os.environ.get("PBX_BENCH_DRYRUN") == "1":  # launcher test: no GPU call
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": world_env,
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}), flush=True)
        return
    # Load libpbx (ROCm 7.2 HIP runtime + RCCL from /opt/rocm) BEFORE torch is
    # imported for the gloo control plane, so torch binds to the same runtime
    # instead of loading its bundled copies under the same sonames.
    nat.load()
    nat.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist = Dist()
    world, rank = dist.world, dist.rank

    from pynbodyext.parallel import ShardedDirect, shard_bounds

    n_tot = args.n_per_gpu * world
    seed = SEEDS.get(n_tot, 1100 + world)
    pos, mass = plummer(n_tot, seed=seed)
    lo, hi = shard_bounds(n_tot, world, rank)
    n_loc = hi - lo
    solver = ShardedDirect(dist.comm, n_tot, pos[lo:hi], mass[lo:hi])

    # one event pair per timed step, read back after the timed region
    events = [(nat.Event(), nat.Event()) for _ in range(args.steps)]
    it = iter(events)

    def step(timed: bool):
        solver.gather_sources()
        if timed:
            e0, e1 = next(it)
            e0.record()
        solver.solve()
        if timed:
            e1.record()

    for _ in range(args.warmup):
        step(False)
    nat.synchronize()
    dist.barrier()
    nat.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    nat.synchronize()
    dist.barrier()
    t1 = time.perf_counter()
    elapsed = dist.max(t1 - t0)
    kernel_ms = [a.elapsed_ms(b) for a, b in events]
    kern_avg_ms = dist.max(float(np.mean(kernel_ms)))

    # the same solve in precise mode (reference arithmetic, direct.rs:173-179:
    # 1/r refined by a Newton step), kernel time only, beside the fast headline
    with nat.precise_mode(True):
        step(False)
        pe = [(nat.Event(), nat.Event()) for _ in range(2)]
        for a, b in pe:
            solver.gather_sources()
            a.record()
            solver.solve()
            b.record()
        nat.synchronize()
    precise_ms = dist.max(float(np.mean([a.elapsed_ms(b) for a, b in pe])))

    pairs_per_step = float(n_tot) * float(n_tot - 1)   # all ranks together
    value = pairs_per_step * args.steps / elapsed
    # roofline: this rank's kernel does n_loc * (n_tot - 1) pairs per launch
    pairs_launch = float(n_loc) * float(n_tot - 1)
    achieved_tf = pairs_launch * FLOP_PER_PAIR / (kern_avg_ms * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic("direct")

    tree = None
    if not args.no_tree:
        tree = bench_tree(dist, args.tree_n, steps=max(3, args.steps), warmup=1,
                          cpu=not args.no_cpu_baseline, cpu_seconds=args.cpu_seconds)
    sweep = None
    if not args.no_profile:
        # every rank: with N > 1 (or PBX_BENCH_FORCE_DIST=1) the sharded
        # profile with global edges (distributed radix select over RCCL)
        sizes = [int(s) for s in args.profile_sizes.split(",") if s]
        # a 1M call is ~0.1 ms: the median of K calls at the bench's default
        # K = 5 moves by +-10 % from run to run, so the profile leg times
        # max(K, 200) calls per size (0.15 s at 64M)
        sweep = bench_profile(sizes, steps=max(200, args.steps), warmup=max(5, args.warmup),
                              cpu=not args.no_cpu_baseline and rank == 0 and world == 1,
                              dist=dist if dist.comm is not None else None)
    api = prof_api = None
    if world == 1 and not args.no_api:
        api = bench_api(pos, mass)
        if not args.no_profile:
            prof_api = bench_profile_api()
    dist.close()
    if rank != 0:
        return
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_rows(cpu_baseline(pos, mass, args.cpu_seconds),
                       cpu_baseline(pos, mass, args.cpu_seconds / 2, cores=1))
    out = {
        "metric": "particle-pairs/sec (direct-sum gravity, force+potential)",
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"{n_tot}-particle Plummer sphere, direct-sum force+potential "
                        f"(Newtonian), {n_loc} targets/GPU x {n_tot} sources"
                        + (", RCCL source all-gather" if world > 1 else ""),
            "n_particles": n_tot,
            "seed": seed,
            "parallelism": f"targets sharded x{world}",
            "device": nat.device_name(),
        },
        "roofline": {
            "bound": "fp64-valu",
            "achieved": achieved_tf,
            "peak": FP64_VECTOR_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tf / FP64_VECTOR_PEAK_TFLOPS,
            "traffic": traffic,
            **{f"precise_{k}": v for k, v in precise_row(pairs_launch * FLOP_PER_PAIR,
                                                          precise_ms).items()
               if k in ("kernel_ms", "achieved", "frac")},
            "traffic_source": traffic_src,
            "kernel": "sym_kernel<pot+acc> (each unordered pair once)" if solver.symmetric else "direct_kernel<Newtonian, pot+acc, self-skip>",
            "mode": "precise" if nat.get_precise() else "fast",
            "flop_per_pair": FLOP_PER_PAIR,
            "kernel_ms": kern_avg_ms,
            **executed_issue(solver.symmetric, pairs_launch, kern_avg_ms),
        },
        "roofline_notes": {
            "mode": "fast: v_rsq_f64 unrefined (~5e-8 per pair, <= 1e-7 vs the oracle); "
                    "precise: + one Newton step (pbx_set_precise); precise_* = the same launch "
                    "in precise mode, not the headline",
            "frac": "algorithmic: 22 flop per ORDERED pair delivered (SURVEY.md §8d)",
            "executed_issue": "FP64 lane-instructions the kernel actually issues / the FP64 VALU "
                              "issue peak (39.3e12/s)"},
        "cpu_baseline": cpu,
        "api_level": api,
    }
    if sweep is not None:
        head = sweep[0]

        def chg(r):  # the changing-input figures of a sweep row (single rank)
            return r.get("changing") or {}

        def rate(r):  # the credited rate: changing inputs where measured
            return chg(r).get("hbm_gbs_algorithmic", r["hbm_gbs_algorithmic_per_gpu"])

        big = max(sweep, key=rate)
        credited = "changing" if chg(big) else "identical"
        # counter-based: the PMC run's HBM bytes per step over this run's stream time
        counter = None
        for r in sweep:
            b, bsrc = pmc_profile_step_bytes(r["n_per_gpu"], credited)
            if b:
                sm = chg(r).get("stream_ms", r["stream_ms"])
                gbs = b / (sm * 1e-3) / 1e9
                counter = {"n_per_gpu": r["n_per_gpu"], "inputs": credited,
                           "hbm_bytes_per_step": b,
                           "achieved_gbs": gbs, "frac_of_spec": gbs / HBM_PEAK_GBS,
                           "frac_of_measured_copy_6290": gbs / 6290.0,
                           "source": f"{bsrc} (2 x FETCH_SIZE + WRITE_SIZE of every profile "
                                     "kernel, per call) / this run's stream_ms"}
        value = chg(head).get("particles_per_s_wall", head["particles_per_s"])
        out["profile"] = {
            "metric": "particles/sec (RadialProfileBuilder equaln 128, Sphere&FamilyFilter, "
                      "weight=mass)",
            "value": value,
            "unit": "particles/s",
            "inputs": ("a different snapshot every call (one handle cycling through "
                       f"{N_CHANGING} snapshots)" if chg(head) else "one snapshot, repeated"),
            "identical_snapshot_value": head["particles_per_s"],
            "config": {"workload": f"{head['n_per_gpu']}-particle Plummer sphere per GPU "
                                   f"(x{world}), Sphere(R=10) & FamilyFilter('dm'), equaln 128 "
                                   "bins, mass sum + mean r"
                                   + (", global edges by distributed radix select"
                                      if world > 1 else ""),
                       "kept_rank0": head["n_kept_rank0"]},
            "scaling": "weak",
            "roofline": {"bound": "hbm", "achieved": rate(big),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": rate(big) / HBM_PEAK_GBS,
                         "inputs": credited,
                         "at_n_per_gpu": big["n_per_gpu"],
                         "stream_ms": chg(big).get("stream_ms", big["stream_ms"]),
                         "identical_snapshot_frac": big["hbm_gbs_algorithmic_per_gpu"] / HBM_PEAK_GBS,
                         "identical_snapshot_stream_ms": big["stream_ms"],
                         "cold_frac": (big["n_per_gpu"] * PROFILE_BYTES_PER_PARTICLE /
                                       (big["cold_stream_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS)
                                      if big.get("cold_stream_ms") else None,
                         "cold_stream_ms": big.get("cold_stream_ms"),
                         "bytes_per_particle": PROFILE_BYTES_PER_PARTICLE,
                         "traffic": pmc_profile_step_bytes(big["n_per_gpu"], credited)[0],
                         "traffic_note": "HBM bytes per call at at_n_per_gpu (all profile "
                                         "kernels: 2 x FETCH_SIZE + WRITE_SIZE, PMC runs "
                                         "committed as profiles/pmc_profile_<N>M.json)"},
            "counter_roofline": counter,
            "by_size": [{"n_per_gpu": r["n_per_gpu"],
                         "changing_stream_ms": chg(r).get("stream_ms"),
                         "changing_frac": chg(r).get("frac"),
                         "cold_stream_ms": r.get("cold_stream_ms"),
                         "identical_stream_ms": r["stream_ms"]} for r in sweep],
            "parity_at_roofline_point": big.get("parity_vs_oracle"),
            "changing_parity_at_roofline_point": chg(big).get("parity"),
            "api_level": prof_api,
            "one_launch_discards": (head.get("path") or {}).get("mono_discarded"),
            "sweep": sweep,
            "cpu_baseline": head.get("cpu_baseline"),
        }
    if tree is not None:
        out["tree"] = tree
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
