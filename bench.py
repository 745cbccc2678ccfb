"""Headline benchmark: prove time + trace rows/s of the 3x3 permutation AIR.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--log-n 19] [--ncols 3]

A "step" is one full ``p3_uni_stark::prove`` (bin/src/main.rs:80-86) of the
3x3 permutation AIR (3 'from' + 3 'to' columns + b_inverse + check, w = 8,
4 quotient chunks, log_blowup 3, 33 queries) on one synthetic 2^log_n-row
trace that is already resident in HBM, ending with the serialized proof on
the host.  For N > 1 (launched by torch.distributed.run) every rank proves its
own independent trace (replicas, no data-path collective);
``value`` = all rows proven by all ranks / the max-over-ranks wall time.

``--shard``: the N ranks prove ONE trace together
(lsp_prove_sharded; rank g owns LDE rows [g N/G, (g+1) N/G)), exchanging
subtree roots, quotient chunks, opened values and query openings over RCCL
(``--comm rccl``, device-direct over xGMI) or a gloo group (``--comm gloo``,
host-staged; lets several ranks share one GPU).  ``value`` = rows of the one
proof / max-over-ranks wall time ("scaling": "strong").

Besides the contract fields the JSON line carries:
  roofline       the coset LDE (the metric's "NTT HBM GB/s"): algorithmic
                 bytes 32*w*(h + N) per coset_lde_batch / its event-timed
                 duration, vs the 8 TB/s HBM3E peak
  roofline_valu  the dominant kernel family (Poseidon2 Merkle hashing):
                 permutations / time vs the permutation rate of the same
                 code on register-resident states (lsp_calibrate_poseidon2)
  cpu_baseline   the C restatement (oracle/, "port") proving a bounded
                 sample on the host cores, rank 0 at N = 1 only
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "prove time (s) + trace-rows/sec, 3x3 perm AIR @2^19; NTT HBM GB/s vs roofline"
PUBLISHED_ROWS_PER_S = 524288 / 330.0  # README.md:11 (~330 s for 2^19 rows, CPU)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-n", type=int, default=19)
    ap.add_argument("--ncols", type=int, default=3)
    ap.add_argument("--air", choices=["perm", "wide"], default="perm",
                    help="perm: the 3x3 permutation AIR (headline); wide: SURVEY 8(d) C3 synthetic "
                         "wide AIR (4 LogUp lookups + 8 permutation groups of 6+6, W = 184)")
    ap.add_argument("--seed", type=int, default=0x4C494E4541)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-log-n", type=int, default=17, help="bounded CPU-baseline sample size")
    ap.add_argument("--shard", action="store_true", help="one proof sharded over the N ranks (C4)")
    ap.add_argument("--comm", choices=["rccl", "gloo"], default="rccl", help="--shard exchange transport")
    ap.add_argument("--device", type=int, default=None, help="GPU of this rank (default: LOCAL_RANK)")
    ap.add_argument("--dump-proof", default=None, help="rank 0 writes the last proof here")
    ap.add_argument("--inflight", type=int, default=3,
                    help="also measure P independent proofs in flight on the GPU (P contexts/streams, "
                         "reported as the separate 'inflight' field, never as value); 0 or 1 disables")
    return ap.parse_args()


def main():
    args = parse()
    from linea_stark_prover_amd.replicas import init_from_env, rank_seed, timed_steps
    dist = init_from_env()  # gloo control plane when WORLD_SIZE > 1 (imports torch first)
    world, rank, local = dist.world, dist.rank, dist.local_rank

    import numpy as np

    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig, gen_permutation_trace, gen_wide_trace

    shard = args.shard
    if shard:
        from linea_stark_prover_amd import shard as S  # imports torch before the HIP library loads
    cfg = StarkConfig(seed=args.seed)
    ctx = Context(cfg, device=local if args.device is None else args.device)
    if shard:
        if args.comm == "rccl":
            S.attach_rccl(ctx)
        else:
            S.GlooComm().attach(ctx)
    a, d, _ = cfg.seeded()
    pub = np.concatenate([a, d])
    h = 1 << args.log_n
    tseed = args.seed if shard else rank_seed(args.seed, rank)  # sharded: every rank holds the same trace
    if args.air == "wide":
        trace, air = gen_wide_trace(args.log_n, a, d, seed=tseed)
    else:
        air = permutation_air(args.ncols)
        trace = gen_permutation_trace(args.log_n, args.ncols, a, d, seed=tseed)
    w = trace.shape[1]
    dtrace = ctx.dev_alloc(trace.nbytes)
    ctx.h2d(dtrace, trace)  # resident in HBM before the timed region

    phases_acc = {}

    def record():
        for name, ms in ctx.last_timings():
            phases_acc[name] = phases_acc.get(name, 0.0) + ms

    if shard:
        step = lambda: S.prove_sharded(ctx, dtrace, air, pub, h, w)  # noqa: E731
    else:
        step = lambda: ctx.prove(dtrace, air, pub, h, w)  # noqa: E731
    elapsed, proof = timed_steps(step, args.steps, args.warmup, dist, sync=ctx.synchronize, on_step=record)
    phases = {k: v / max(args.steps, 1) for k, v in phases_acc.items()}
    verified = ctx.verify(proof, air, pub) if proof is not None else False

    if rank == 0 and args.dump_proof and proof is not None:
        with open(args.dump_proof, "wb") as f:
            f.write(proof)
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = (1 if shard else world) * h * args.steps / elapsed
        N = h << cfg.log_blowup
        import ctypes
        from linea_stark_prover_amd import _lib
        desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
        lq = ctypes.c_uint32()
        _lib.check(_lib.lib().lsp_log_quotient_degree(desc, len(desc), cfg.public_degree, ctypes.byref(lq)))
        q = 1 << lq.value
        lde_ms = phases.get("coset_lde_batch", float("nan"))
        Nr = N // world if shard else N  # LDE rows (Merkle leaves) this rank computes
        lde_bytes = 32 * w * (h + Nr)
        achieved = lde_bytes / (lde_ms * 1e-3) / 1e9
        merkle_ms = phases.get("merkle tree", float("nan"))
        trace_perms = Nr * ((w + 1) // 2) + (Nr - 1)
        calib = ctx.calibrate_poseidon2()
        valu_achieved = trace_perms / (merkle_ms * 1e-3) / 1e6
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "trace-rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "prove_time_s": ms_per_step / 1e3,
            "higher_is_better": True,
            "scaling": "strong" if shard else "weak",
            "vs_baseline": value / PUBLISHED_ROWS_PER_S,
            "baseline_published": {"value": PUBLISHED_ROWS_PER_S, "unit": "trace-rows/s",
                                   "source": "reference README.md:11, ~330 s for 2^19 rows on a 16-core CPU"},
            "dtype": "fr253 (BLS12-377 Fr, 8x u32 Montgomery limbs)",
            "data": "synthetic (seeded permutation trace, SURVEY 8(d) " + ("C4)" if shard else "C1)"),
            "config": {"workload": (f"{args.ncols}x{args.ncols} permutation AIR" if args.air == "perm" else
                                    "wide AIR (4 LogUp lookups + 8 permutation groups of 6+6)") +
                                   f", 2^{args.log_n} rows (w={w}, q={q} quotient chunks, log_blowup "
                                   f"{cfg.log_blowup}, {cfg.num_queries} queries, Poseidon2-w3 Merkle, FRI)",
                       "log_n": args.log_n, "width": w, "fri_queries": cfg.num_queries,
                       "parallelism": (f"sharded{world} ({args.comm})" if shard else
                                       "replicas" if world > 1 else "single-gpu")},
            "verified": bool(verified),
            "phases_ms": {k: round(v, 3) for k, v in phases.items()},
            "roofline": {"bound": "hbm", "kernel": "coset_lde_batch (trace, w x 2^log_n -> 8x)",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": lde_traffic(args.log_n, w),
                         "valu_issue": valu_issue(["k_ntt_rm"]),
                         "note": "VALU-bound: valu_issue = share of the chip's VALU issue slots the NTT passes "
                                 "use (PMC, profiles/*_valu_pmc.json); HBM frac is low by design",
                         "algorithmic_bytes": lde_bytes, "ms": lde_ms},
            "roofline_valu": {"bound": "valu", "kernel": "trace Merkle tree (Poseidon2 leaf hash + levels)",
                              "achieved": valu_achieved, "unit": "M perm/s",
                              "peak": calib, "frac": valu_achieved / calib,
                              "peak_source": "lsp_calibrate_poseidon2: register-resident chained permutations",
                              "valu_issue": valu_issue(["k_hash_rows1<11u, false>", "k_merkle_level<11u, false>"]),
                              "perms": trace_perms, "fr_mul_per_perm": 230, "ms": merkle_ms},
        }
        if world == 1 and not shard and args.inflight > 1:
            out["inflight"] = inflight(args, cfg, air, pub, trace, ctx, dtrace)
        if world == 1 and not args.no_cpu_baseline and args.air == "perm":
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    ctx.dev_free(dtrace)
    ctx.close()
    dist.close()


def inflight(args, cfg, air, pub, trace, ctx, dtrace):
    """Production throughput mode: P independent proofs in flight on one GPU
    (P contexts = P HIP streams, one host thread each), so one proof's
    latency-bound phases (narrow Merkle levels, transcript, tree tops) overlap
    another's hashing.  Reported beside `value` (the sequential single-proof
    rate), never instead of it."""
    import threading
    from linea_stark_prover_amd.prover import Context
    P, K = args.inflight, max(args.steps, 2)
    h, w = trace.shape[0], trace.shape[1]
    ctxs, ptrs = [ctx], [dtrace]
    for _ in range(P - 1):
        c = Context(cfg, device=ctx_device(ctx, args))
        p = c.dev_alloc(trace.nbytes)
        c.h2d(p, trace)
        c.prove(p, air, pub, h, w)  # warm
        ctxs.append(c)
        ptrs.append(p)
    for c in ctxs:
        c.synchronize()

    def worker(i):
        for _ in range(K):
            ctxs[i].prove(ptrs[i], air, pub, h, w)

    t = time.perf_counter()
    th = [threading.Thread(target=worker, args=(i,)) for i in range(P)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t
    for c, p in zip(ctxs[1:], ptrs[1:]):
        c.dev_free(p)
        c.close()
    return {"proofs_in_flight": P, "proofs": P * K, "value": P * K * h / dt, "unit": "trace-rows/s",
            "ms_per_proof": dt / (P * K) * 1e3,
            "note": "independent proofs on P streams of one GPU; value above is one proof at a time"}


def ctx_device(ctx, args):
    return int(os.environ.get("LOCAL_RANK", "0")) if args.device is None else args.device


def valu_issue(kernels):
    """Calls-weighted VALU issue utilisation of the named kernels from the
    committed PMC passes (tools/pmc_valu.sh -> profiles/*_valu_pmc.json, 2^19
    prove): SQ_INSTS_VALU * 4 / (1024 SIMDs * cycles); None if absent."""
    import glob
    d = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu_pmc.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
    if not d:
        return None
    ks = [v for k, v in d["kernels"].items() if any(k.startswith(p) for p in kernels)]
    ms = sum(v["ms"] for v in ks)
    return round(sum(v["valu_issue"] * v["ms"] for v in ks) / ms, 3) if ms else None


def lde_traffic(log_n, w):
    """HBM bytes per coset_lde_batch from the rocprofv3 PMC passes of
    tools/pmc_round.sh (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction), kept in
    profiles/; None when no measurement matches this size."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_lde_traffic.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("h") == (1 << log_n) and d.get("w") == w:
            best = d["traffic_bytes"]
    return best


def cpu_baseline(args):
    """The oracle's C restatement proving a bounded sample of the same workload
    on the host (test infrastructure used only as the reported baseline)."""
    from oracle import cref
    cref.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    p = cref.setup(args.seed)
    tb, w = cref.gen_perm_trace(p, args.cpu_log_n, args.ncols, seed=args.seed)
    t = time.perf_counter()
    cref.prove(p, tb, 1 << args.cpu_log_n, w, cref.perm_air(args.ncols), nthreads=threads)
    dt = time.perf_counter() - t
    return {"value": (1 << args.cpu_log_n) / dt, "unit": "trace-rows/s", "cores": threads, "kind": "port",
            "seconds": dt,
            "sample": f"oracle/lsp_oracle.c full prove, {args.ncols}x{args.ncols} permutation AIR at "
                      f"2^{args.cpu_log_n} rows (same conventions/seed), {threads} threads"}


if __name__ == "__main__":
    main()
