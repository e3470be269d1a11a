"""Two ranks of the distributed radial profile on ONE GPU (a rehearsal of
the multi-GPU path: RCCL may refuse two ranks on one device — then this
prints the error and exits 3).  Each rank holds half of a particle set;
rank 0 checks the global edges / counts / sums against the oracle on the
whole set.  usage: python tools/two_rank_profile.py [n] (spawns its ranks)"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "pynbody-extras_amd")]


def rank_main(rank, world, n):
    import numpy as np

    from pynbodyext import _native as nat
    from pynbodyext.parallel import Communicator, FileRendezvous, ShardedProfile
    from pynbodyext.profiles._device import SRC_NONE, SRC_W, SRC_X, DeviceBins
    from pynbodyext.synthetic import plummer

    nat.load()
    nat.set_device(0)
    rdzv = FileRendezvous(rank, world, key=os.environ["PBX_TR_KEY"])
    uid = rdzv.broadcast(Communicator.unique_id() if rank == 0 else None)
    comm = Communicator(world, rank, uid)
    pos, mass = plummer(n, seed=77)
    lo, hi = (n * rank) // world, (n * (rank + 1)) // world
    stats = [(SRC_W, SRC_NONE, 1 << 3), (SRC_X, SRC_W, 0b11)]
    out = {}
    for case, kw in [("plain", {}), ("sphere", {"sphere": ((0.0, 0.0, 0.0), 5.0)}),
                     ("clip", {"bin_min": 0.1, "bin_max": 3.0})]:
        dev = DeviceBins()
        sp = ShardedProfile(comm, dev, offset=lo)
        e, c, m = sp.radial_equaln(pos[lo:hi], mass[lo:hi], nbins=128, stats=stats, **kw)
        res = {"edges": e.tolist(), "counts": c.tolist(), "msum": m[0][:, 3].tolist(),
               "local": dev.counts.tolist()}
        dev.close()
        out[case] = res
    comm.barrier()
    if rank == 0:
        from oracle import profile_ref as pr

        ok = True
        for case, kw in [("plain", {}), ("sphere", {"sphere": ((0.0, 0.0, 0.0), 5.0)}),
                         ("clip", {"bin_min": 0.1, "bin_max": 3.0})]:
            keep = np.ones(n, bool)
            if "sphere" in kw:
                keep = pr.sphere_mask(pos, 5.0)
            x, w = pr.radial_r(pos[keep]), mass[keep]
            edges = pr.edges_equaln(x, 128, kw.get("bin_min"), kw.get("bin_max"))
            perm, offs, cnt = pr.assign(x, edges)
            ms, _ = pr.compute(w, w, perm, offs, "sum")
            r = out[case]
            ge, gc = np.array(r["edges"]), np.array(r["counts"])
            gm = np.array(r["msum"])
            okc = (np.array_equal(ge, edges) and np.array_equal(gc, cnt)
                   and np.nanmax(np.abs(gm - ms) / np.abs(ms)) < 1e-12)
            print(json.dumps({"case": case, "edges": bool(np.array_equal(ge, edges)),
                              "counts": bool(np.array_equal(gc, cnt)),
                              "msum_rel": float(np.nanmax(np.abs(gm - ms) / np.abs(ms)))}))
            ok &= okc
        print("TWO_RANK_OK" if ok else "TWO_RANK_MISMATCH", flush=True)
    comm.destroy()
    rdzv.cleanup()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--rank":
        rank_main(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
        sys.exit(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
    env = dict(os.environ, PBX_TR_KEY=f"tr{os.getpid()}", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, __file__, "--rank", str(r), "2", str(n)], env=env)
             for r in range(2)]
    rc = [p.wait(timeout=120) for p in procs]
    sys.exit(max(rc))
