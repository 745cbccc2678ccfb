"""One rank of a G-rank sharded proof, rehearsed on a single GPU.

    python tools/rank_rehearsal.py [--log-n 26] [--size 8] [--ranks 0,7] [--steps 2]

BASELINE configs[3] (the 3x3 permutation AIR at 2^26 rows over 8 MI355X) needs
8 GPUs; this box has one.  Each listed rank g runs in its own child process
(a fresh device and pool): it proves the full-size trace as rank g of G with
the loopback transport (lsp_ctx_attach_loopback: peers' parts of each exchange
fabricated locally), so its device memory and per-phase times are rank g's
at the real shapes.  The proof is not valid (the library refuses to serialize
it; only its wire size is read, which must be the real proof's).  Prints one
JSON object per rank: wall time per step, the phase times of the last step,
the context's pool (the high-water mark of its working set), the GPU's used
memory against its total, the proof's wire size and the collective schedule
the rank issued (lsp_comm_log: op, bytes, root, what it carried, device ms).
tests/test_gpu_configs_full.py runs it at BASELINE configs[3]'s size.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one_rank(log_n, rank, size, steps, ncols=3):
    import ctypes

    import numpy as np

    from linea_stark_prover_amd import _lib as L
    from linea_stark_prover_amd import shard as S  # torch first: one HIP runtime
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig

    cfg = StarkConfig()
    a, d, _ = cfg.seeded()
    pub = np.concatenate([a, d])
    air = permutation_air(ncols)
    h, w = 1 << log_n, 2 * ncols + 2
    ctx = Context(cfg)
    L.check(L.lib().lsp_ctx_attach_loopback(ctx.h, rank, size), ctx.h)

    def mem():
        pool, used, tot = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        ctx._chk(L.lib().lsp_ctx_mem_stats(ctx.h, ctypes.byref(pool), ctypes.byref(used), ctypes.byref(tot)))
        return pool.value, used.value, tot.value

    t = time.perf_counter()
    dtrace = ctx.gen_permutation_trace_device(log_n, ncols, a, d)
    ctx.synchronize()
    gen_s = time.perf_counter() - t
    nbytes = S.prove_sharded(ctx, dtrace, air, pub, h, w, size_only=True)  # warm-up: pool, tables
    ts = []
    for _ in range(steps):
        ctx.synchronize()
        t = time.perf_counter()
        nbytes = S.prove_sharded(ctx, dtrace, air, pub, h, w, size_only=True)
        ctx.synchronize()
        ts.append(time.perf_counter() - t)
    phases = {k: round(v, 3) for k, v in ctx.last_timings()}
    sched, _ = ctx.comm_log()
    try:  # a rehearsal proof is refused as bytes: the library marks it
        S.prove_sharded(ctx, dtrace, air, pub, h, w)
        refused = False
    except L.LspError as e:
        refused = e.code == L.LSP_E_STATE
    pool, used, tot = mem()
    trace_bytes = h * w * 32
    return {"log_n": log_n, "rank": rank, "size": size, "steps": steps, "step_s": [round(x, 4) for x in ts],
            "prove_s_median": sorted(ts)[len(ts) // 2], "trace_gen_s": round(gen_s, 3), "phases_ms": phases,
            "trace_bytes": trace_bytes, "pool_bytes": pool, "device_used_bytes": used, "device_total_bytes": tot,
            "pool_plus_trace_gib": round((pool + trace_bytes) / 2**30, 2), "device_used_gib": round(used / 2**30, 2),
            "fits_288gb": used < 288e9, "proof_wire_bytes": nbytes, "rehearsal_bytes_refused": refused,
            "comm_log": sched}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=26)
    ap.add_argument("--size", type=int, default=8)
    ap.add_argument("--ranks", default="0,7")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--one", type=int, default=None, help=argparse.SUPPRESS)  # child: run this rank
    a = ap.parse_args()
    if a.one is not None:
        print(json.dumps(one_rank(a.log_n, a.one, a.size, a.steps)), flush=True)
        return 0
    for r in [int(x) for x in a.ranks.split(",")]:
        # a child process per rank: a fresh device and pool (the parent never touches the GPU)
        cmd = [sys.executable, os.path.abspath(__file__), "--log-n", str(a.log_n), "--size", str(a.size),
               "--steps", str(a.steps), "--one", str(r)]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            sys.stderr.write(p.stderr[-4000:])
            return p.returncode
        print(p.stdout.strip().splitlines()[-1], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
