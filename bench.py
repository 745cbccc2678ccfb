"""Headline benchmark: prove time + trace rows/s of the 3x3 permutation AIR.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--log-n 19] [--ncols 3]

A "step" is one full ``p3_uni_stark::prove`` (bin/src/main.rs:80-86) of the
3x3 permutation AIR (3 'from' + 3 'to' columns + b_inverse + check, w = 8,
4 quotient chunks, log_blowup 3, 33 queries) on one synthetic 2^log_n-row
trace that is already resident in HBM, ending with the serialized proof on
the host.

Ranks.  ``--gpus N`` with N > 1 needs N processes: under
torch.distributed.run (WORLD_SIZE set) every process is one rank; started
without a launcher, bench.py starts ``torch.distributed.run --nproc-per-node
N`` itself as a child process (before anything touches the GPU) and exits with
its status.  WORLD_SIZE != --gpus is an error, never a silent single rank.

Legs (rank 0 prints ONE JSON line):
  value          C5 replicas: every rank proves its own
                 independent 2^log_n trace, no data-path collective; value =
                 all rows / max-over-ranks wall time ("scaling": "weak").
                 ``--shard`` instead proves ONE trace over the N ranks
                 (lsp_prove_sharded, "scaling": "strong").
  batch          BASELINE configs[4] (configs[1] at N = 1): every rank proves
                 its own 2^22-row trace (device-generated); all rows / the
                 slowest rank's time (--batch-leg).
  sharded        C4 (BASELINE configs[3]): one 2^24-row proof
                 sharded over all N ranks (rank g owns LDE rows
                 [g N/G, (g+1) N/G)), exchanging subtree roots, quotient
                 chunks, opened values and query openings over RCCL (one GPU
                 per rank) or gloo (ranks sharing a GPU); at N = 8 also
                 2^26.  The trace is generated on every GPU from the same
                 seed (lsp_gen_permutation_trace_device).  At N = 1 it is
                 lsp_prove itself: prove_shard over the one-rank SoloComm.
                 A per-rank watchdog bounds the leg (--shard-timeout).
  prove_time_host_trace_s   (N = 1) the same proof with the trace uploaded
                 from host memory inside every step (SURVEY 8(d) "H2D
                 included"); mean and median.
  roofline       the coset LDE (the metric's "NTT HBM GB/s"): algorithmic
                 bytes 32*w*(h + N) per coset_lde_batch / its event-timed
                 duration, vs the 8 TB/s HBM3E peak
  roofline_valu  the dominant kernel family (Poseidon2 Merkle hashing):
                 permutations / time vs the chip's peak permutation rate
                 from the measured v_mad_u64_u32 issue rate
                 (profiles/r02_rates.json, tools/ubench/rates.hip): 230
                 Fr-muls x 128 MADs per permutation
  cpu_baseline   the C restatement (oracle/, "port") proving the headline
                 2^19 workload on the host cores, rank 0 at N = 1 only
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "prove time (s) + trace-rows/sec, 3x3 perm AIR @2^19; NTT HBM GB/s vs roofline"
PUBLISHED_ROWS_PER_S = 524288 / 330.0  # README.md:11 (~330 s for 2^19 rows, CPU)
HBM_PEAK_GBS = 8000.0
RATES_FILE = os.path.join(ROOT, "profiles", "r02_rates.json")
NOMINAL_GHZ = 2.4           # MI355X peak engine clock (MI355X_MICROARCH.md)
SIMDS = 256 * 4             # 256 CUs x 4 SIMD-32 units
FR_MUL_PER_PERM = 230       # 46 S-boxes x 5 products (x^11), SURVEY 8 conventions
MAD_PER_FR_MUL = 128        # 8 x 32-bit limbs: 64 product + 64 reduction MADs (the floor the peak assumes)
FRMUL_PEAK_GPS = SIMDS * 64 / 4 * NOMINAL_GHZ / MAD_PER_FR_MUL  # 307.2 G Fr-mul/s (v_mad_u64_u32: 4 cycles)


class ClockSampler:
    """The engine clock the SMU reports while the timed steps run (VERDICT r5
    item 1: a box-speed stamp, so lines from different boxes can be told
    apart from code changes).  A thread reads amdsmi's gpu_metrics every
    `period` s between start() and stop(): current_gfxclk(s) (per XCD on
    MI355X; their mean), average_gfxclk_frequency and socket power.  Read-only
    sysfs queries; the device is matched by PCI bus id.  Absent amdsmi or a
    device it cannot see, `status` says why and summary() is None."""

    def __init__(self, hip_device: int, period: float = 0.02):
        self.period, self.samples, self.handle, self.bdf = period, [], None, None
        self.status, self._stop, self._th = "ok", threading.Event(), None
        try:
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            buf = ctypes.create_string_buffer(64)
            if hip.hipDeviceGetPCIBusId(buf, 64, ctypes.c_int(hip_device)) != 0:
                raise RuntimeError("hipDeviceGetPCIBusId failed")
            self.bdf = buf.value.decode().lower()
            import amdsmi
            amdsmi.amdsmi_init()
            handles = amdsmi.amdsmi_get_processor_handles()
            for hd in handles:
                if amdsmi.amdsmi_get_gpu_device_bdf(hd).lower() == self.bdf:
                    self.handle = hd
            if self.handle is None and len(handles) == 1:
                self.handle = handles[0]
            if self.handle is None:
                self.status = f"no amdsmi device with bus id {self.bdf} among {len(handles)}"
            else:
                self._read()  # fails here, not in the thread
        except Exception as e:  # noqa: BLE001  (a stamp, never a reason to fail the bench)
            self.status, self.handle = f"{type(e).__name__}: {e}", None

    def _read(self):
        import amdsmi
        m = amdsmi.amdsmi_get_gpu_metrics_info(self.handle)
        clks = m.get("current_gfxclks")
        clks = [c for c in clks if isinstance(c, (int, float)) and c > 0] if isinstance(clks, list) else []
        cur = statistics.mean(clks) if clks else m.get("current_gfxclk")
        num = lambda v: float(v) if isinstance(v, (int, float)) else None  # noqa: E731
        return (num(cur), num(m.get("average_gfxclk_frequency")), num(m.get("current_socket_power")))

    def _run(self):
        while not self._stop.wait(self.period):
            try:
                self.samples.append(self._read())
            except Exception:  # noqa: BLE001
                pass

    def start(self):
        if self.handle is not None:
            self.samples, self._stop = [], threading.Event()
            self._th = threading.Thread(target=self._run, daemon=True)
            self._th.start()
        return self

    def stop(self):
        if self._th is not None:
            self._stop.set()
            self._th.join()
            self._th = None
        return self.summary()

    def summary(self):
        cur = [s[0] for s in self.samples if s[0]]
        if not cur:
            return None
        avg = [s[1] for s in self.samples if s[1]]
        pw = [s[2] for s in self.samples if s[2]]
        return {"sclk_mhz_mean": statistics.mean(cur), "sclk_mhz_median": statistics.median(cur),
                "sclk_mhz_min": min(cur), "sclk_mhz_max": max(cur),
                "avg_gfxclk_mhz_mean": statistics.mean(avg) if avg else None,
                "socket_power_w_mean": statistics.mean(pw) if pw else None,
                "samples": len(cur), "period_s": self.period}




def box_speed(ctx, sclk, status, ms_per_step):
    """What this box did while the line was measured, beside the line: the
    engine clock during the timed steps (ClockSampler), the GPU's
    full-occupancy Poseidon2 rate (k_calib_perm, best of 2..32 waves per SIMD)
    and one host thread's Poseidon2 compression rate (the tree tops' and FRI
    tail's path).  Lines from two boxes compare by these, not by assumption."""
    out = {"gpu_perm_mperm_per_s": ctx.calibrate_poseidon2(),
           "gpu_perm_note": "k_calib_perm over 2..32 waves per SIMD (best): a full-occupancy throughput probe "
                            "of the permutation every Merkle kernel runs",
           "host_compress_k_per_s": host_compress_rate(ctx) / 1e3,
           "host_compress_note": "lsp_host_compress_batch, one thread, 4096 compressions, best of 5",
           "sclk_during_timed_steps": sclk, "sclk_status": status}
    if sclk:
        out["ms_per_step_x_sclk_ghz"] = ms_per_step * sclk["sclk_mhz_mean"] / 1e3
    return out


def host_compress_rate(ctx, n: int = 4096, reps: int = 5) -> float:
    """Host Poseidon2 compressions per second on one thread (lsp_host_compress_batch:
    the IFMA path the tree tops and the FRI tail run on), best of `reps`: the
    host half of the box-speed stamp."""
    import ctypes
    import numpy as np
    from linea_stark_prover_amd import _lib
    rng = np.random.default_rng(7)
    pairs = np.ascontiguousarray(rng.integers(0, 1 << 60, size=(2 * n, 4), dtype=np.uint64))  # < 2^252 < r
    out = np.zeros((n, 4), dtype=np.uint64)
    best = 0.0
    for _ in range(reps):
        t = time.perf_counter()
        _lib.check(_lib.lib().lsp_host_compress_batch(ctx.h, pairs.ctypes.data_as(_lib.c_fr_p), n,
                                                      out.ctypes.data_as(_lib.c_fr_p)))
        best = max(best, n / (time.perf_counter() - t))
    return best


def _lib_src() -> str:
    """the stamp of the library being benched (build.library_hash); the
    working tree's hash only for an unstamped library"""
    from linea_stark_prover_amd.build import library_hash, source_hash
    return library_hash() or source_hash()


ROOFLINE_PHASES = ("coset_lde_batch", "merkle tree")  # the phases `roofline` / `roofline_valu` time
LIB_SRC = _lib_src()  # the build the committed PMC profiles must match
VALU_SRC, TRAFFIC_SRC = {}, {}  # where each PMC-derived field came from (or why it is null)


def lde_products(h: int, w: int, ncosets: int) -> int:
    """algorithmic Fr products of one coset LDE of an h x w matrix into
    ncosets cosets of h: the inverse NTT, one twist per coefficient and coset,
    and one forward NTT of h per coset"""
    lg = h.bit_length() - 1
    return w * ((h // 2) * lg + ncosets * h + ncosets * (h // 2) * lg)


def parse(argv=None):
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
    ap.add_argument("--cpu-log-n", type=int, default=None,
                    help="CPU-baseline size (rows = 2^cpu_log_n; default: the headline's --log-n, BASELINE.md's "
                         "2^19 input)")
    ap.add_argument("--cpu-runs", type=int, default=5, help="CPU-baseline timed runs (median; BASELINE.md's plan: 5)")
    ap.add_argument("--cpu-warmup", type=int, default=1,
                    help="untimed CPU-baseline runs first (BASELINE.md's plan: 1; about 10 s each at 2^19)")
    ap.add_argument("--cpu-small-log-n", type=int, default=0,
                    help="an extra, smaller CPU sample reported beside the headline one (0, the default, disables: "
                         "the headline-size sample is the baseline)")
    ap.add_argument("--wide-leg", type=int, default=20,
                    help="log2 rows of the wide_c3 leg (BASELINE configs[2], the synthetic wide AIR, W = 184); "
                         "0 skips")
    ap.add_argument("--wide-steps", type=int, default=3, help="timed proofs of the wide_c3 leg (median)")
    ap.add_argument("--shape-leg", default="6",
                    help="ncols of the extra 2^log_n leg in bench.log's shape (6+6 columns, w = 14, the "
                         "reference's only measured run, bench.log:18-20); 'none' to skip")
    ap.add_argument("--shape-pow-bits", type=int, default=29,
                    help="the shape leg once more with this many proof-of-work bits (29: bench.log's run, which "
                         "ground a witness, bench.log:65, 19.3 s; bin/src/main.rs:62 sets 0 with the comment "
                         "//29); 0 skips")
    ap.add_argument("--shard", action="store_true", help="main leg: one proof sharded over the N ranks (C4)")
    ap.add_argument("--comm", choices=["rccl", "gloo"], default="rccl", help="--shard exchange transport")
    ap.add_argument("--shard-leg", default="auto",
                    help="C4 'sharded' leg sizes, comma-separated log2 rows; 'auto' = 24 (and 26 at N = 8); "
                         "'none' disables")
    ap.add_argument("--shard-leg-steps", type=int, default=2)
    ap.add_argument("--shard-leg-warmup", type=int, default=1)
    ap.add_argument("--shard-comm", choices=["auto", "rccl", "gloo"], default="auto",
                    help="auto: RCCL when every rank has its own GPU, else gloo")
    ap.add_argument("--shard-timeout", type=float, default=240.0,
                    help="seconds before a rank's watchdog abandons the sharded leg (the 2^24 and 2^26 legs "
                         "take well under a minute on 8 GPUs; a hung first multi-rank RCCL run must still "
                         "leave time for the main line inside a driver's bench budget)")
    ap.add_argument("--no-host-trace-leg", action="store_true")
    ap.add_argument("--batch-leg", default="22",
                    help="log_n list of the batch leg (BASELINE configs[4]: one independent 2^22 proof per "
                         "GPU; at N = 1 configs[1]); 'none' to skip")
    ap.add_argument("--batch-leg-steps", type=int, default=2)
    ap.add_argument("--device", type=int, default=None, help="GPU of this rank (default: LOCAL_RANK mod #GPUs)")
    ap.add_argument("--dump-proof", default=None, help="rank 0 writes the last proof here")
    ap.add_argument("--dump-batch-proofs", default=None,
                    help="every rank writes its batch-leg proof to <this>.<rank>.<log_n>.bin")
    ap.add_argument("--dump-comm-schedule", default=None,
                    help="--shard --comm gloo: every rank writes the collectives its communicator carried, in "
                         "order, to <this>.<rank>.json")
    ap.add_argument("--inflight", type=int, default=3,
                    help="also measure P independent proofs in flight on the GPU (P contexts/streams, "
                         "reported as the separate 'inflight' field, never as value); 0 or 1 disables")
    ap.add_argument("--dry-run", action="store_true",
                    help="set up the ranks and the control group, print the rank census, no GPU work")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """--gpus N > 1 without a launcher: run N ranks under torch.distributed.run
    as a child process (nothing here has touched the GPU) and return its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(json.dumps({"error": f"WORLD_SIZE={world_env} but --gpus {args.gpus}: refusing to report "
                                   f"{world_env} rank(s) as {args.gpus} GPU(s)"}), flush=True)
        return 2
    from linea_stark_prover_amd.replicas import init_from_env
    dist = init_from_env()  # gloo control plane when WORLD_SIZE > 1 (imports torch first)
    world, rank = dist.world, dist.rank
    ranks_seen = int(round(dist.sum(1.0)))
    if args.dry_run:
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "n_ranks_seen": ranks_seen,
                              "launcher": "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ
                              else "env"}), flush=True)
        dist.close()
        return 0

    shard_sizes = shard_leg_sizes(args, world)
    if args.shard or (shard_sizes and world > 1):
        from linea_stark_prover_amd import shard as S  # noqa: F401  (torch before the HIP library)
    out, ctx = main_leg(args, dist, ranks_seen)
    batch_sizes = [] if args.batch_leg == "none" or args.shard or args.air != "perm" else \
        [int(x) for x in args.batch_leg.split(",") if x]
    if batch_sizes:
        try:
            batch = batch_leg(args, dist, ctx, batch_sizes)
        except Exception as e:  # the main line is still reported
            batch = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            out["batch"] = batch
    if world == 1 and args.wide_leg > 0 and args.air == "perm" and not args.shard:
        try:
            out["wide_c3"] = wide_leg(args, dist, ctx, args.wide_leg)
        except Exception as e:  # the main line is still reported
            out["wide_c3"] = {"error": f"{type(e).__name__}: {e}"}
    if world == 1 and args.shape_leg != "none" and args.air == "perm" and not args.shard:
        try:
            out["shape_bench_log"] = shape_leg(args, dist, ctx, int(args.shape_leg))
        except Exception as e:  # the main line is still reported
            out["shape_bench_log"] = {"error": f"{type(e).__name__}: {e}"}
    if shard_sizes:
        sharded = guarded_shard_leg(args, dist, ctx, shard_sizes, out)
        if rank == 0:
            out["sharded"] = sharded
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline and args.air == "perm":
            cb = cpu_baseline(args)
            if cb["log_n"] == args.log_n:
                cb["gpu_speedup"] = out["value"] / cb["value"]
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    ctx.close()
    dist.close()
    return 0


def device_of(args, dist) -> int:
    if args.device is not None:
        return args.device
    import ctypes
    from linea_stark_prover_amd import _lib
    n = ctypes.c_int()
    _lib.check(_lib.lib().lsp_device_count(ctypes.byref(n)))
    return dist.local_rank % max(n.value, 1)


def main_leg(args, dist, ranks_seen):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig, gen_permutation_trace, gen_wide_trace
    from linea_stark_prover_amd.replicas import rank_seed, timed_steps
    import numpy as np

    world, rank = dist.world, dist.rank
    shard = args.shard
    cfg = StarkConfig(seed=args.seed)
    ctx = Context(cfg, device=device_of(args, dist))
    # timed proofs record device events only for the phases the roofline
    # objects read; the full phase breakdown comes from one extra proof after
    # the timed steps (every phase event costs host API time inside the step)
    ctx.set_phase_timing(True, only=ROOFLINE_PHASES)
    if shard:
        from linea_stark_prover_amd import shard as S
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

    phases_acc, step_s = {}, []

    def record():
        for name, ms in ctx.last_timings():
            phases_acc[name] = phases_acc.get(name, 0.0) + ms

    if shard:
        from linea_stark_prover_amd import shard as S
        step = lambda: S.prove_sharded(ctx, dtrace, air, pub, h, w)  # noqa: E731
    else:
        step = lambda: ctx.prove(dtrace, air, pub, h, w)  # noqa: E731
    clocks = ClockSampler(ctx.device)
    elapsed, proof = timed_steps(step, args.steps, args.warmup, dist, sync=ctx.synchronize, step_times=step_s,
                                 on_start=clocks.start)
    sclk = clocks.stop()
    # the last timed step's LDE and Merkle times (HIP events on the prover's
    # stream, inside the timed region): the library resolves its phase events
    # lazily, so reading them after every step would put that inside the timing
    record()
    roof_phases = dict(phases_acc)
    # every phase, from one more (untimed) proof
    ctx.set_phase_timing(True)
    step()
    phases_acc.clear()
    record()
    phases = dict(phases_acc)
    ctx.set_phase_timing(True, only=ROOFLINE_PHASES)
    verified = ctx.verify(proof, air, pub) if proof is not None else False
    if rank == 0 and args.dump_proof and proof is not None:
        with open(args.dump_proof, "wb") as f:
            f.write(proof)
    # one process per rank: every collective of the last proof, per rank (lsp_comm_log)
    table = collective_table(ctx, dist) if shard and world > 1 else None
    comm = getattr(ctx, "_comm", None)
    if args.dump_comm_schedule and comm is not None:
        with open(f"{args.dump_comm_schedule}.{rank}.json", "w") as f:
            json.dump({"rank": rank, "world": world, "schedule": comm.schedule}, f)

    out = None
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = (1 if shard else world) * h * args.steps / elapsed
        N = h << cfg.log_blowup
        q = 1 << air_log_q(air, cfg)
        lde_ms = roof_phases.get("coset_lde_batch", float("nan"))
        Nr = N // world if shard else N  # LDE rows (Merkle leaves) this rank computes
        lde_bytes = 32 * w * (h + Nr)
        achieved = lde_bytes / (lde_ms * 1e-3) / 1e9
        lde_frmul = lde_products(h, w, Nr // h)
        frmul_gps = lde_frmul / (lde_ms * 1e-3) / 1e9
        merkle_ms = roof_phases.get("merkle tree", float("nan"))
        trace_perms = Nr * ((w + 1) // 2) + (Nr - 1)
        valu_achieved = trace_perms / (merkle_ms * 1e-3) / 1e6
        peak = valu_peak()
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "trace-rows/s",
            "n_gpus": world,
            "n_ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "prove_time_s": ms_per_step / 1e3,
            "prove_time_median_s": statistics.median(step_s) if step_s else None,
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
                                       f"replicas{world}" if world > 1 else "single-gpu")},
            "verified": bool(verified),
            "phases_ms": {k: round(v, 3) for k, v in phases.items()},
            "phases_source": "one untimed proof after the timed steps; the timed steps time only "
                             + " and ".join(ROOFLINE_PHASES) + " (the roofline objects' ms)",
            "lib_src_sha16": LIB_SRC,
            "host_threads": ctx.host_threads(),
            "roofline": {"bound": "hbm", "kernel": "coset_lde_batch (trace, w x 2^log_n -> 8x)",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": lde_traffic(args.log_n, w),
                         "traffic_source": TRAFFIC_SRC.get((args.log_n, w)),
                         "valu_issue": valu_issue(["k_ntt_rm"]),
                         "valu_issue_source": VALU_SRC.get("src"),
                         "frmul_frac": frmul_gps / FRMUL_PEAK_GPS,
                         "frmul": {"products_per_call": lde_frmul, "achieved_g_per_s": frmul_gps,
                                   "peak_g_per_s": FRMUL_PEAK_GPS,
                                   "count": "w x [(h/2) log2 h (inverse) + N (coset twists) + (N/2) log2 h "
                                            "(8 forward coset NTTs of h)] Fr products",
                                   "peak_basis": "1024 SIMDs x 64 lanes / 4 cycles per v_mad_u64_u32 x 2.4 GHz / "
                                                 "128 MADs per 8 x 32-bit Montgomery product",
                                   "impl_mad_floor": ntt_impl_floor(frmul_gps, peak)},
                         "limiter": "valu",
                         "note": "bound/frac are against HBM, the roofline the metric names (NTT HBM GB/s); the "
                                 "kernel itself is limited by the integer VALU, not HBM (limiter): valu_issue = share "
                                 "of SIMD cycles issuing VALU in the NTT passes (PMC SQ_ACTIVE_INST_VALU, "
                                 "profiles/*_valu_pmc.json), frmul_frac = its Fr products against the 128-MAD peak",
                         "algorithmic_bytes": lde_bytes, "ms": lde_ms},
            "roofline_valu": {"bound": "valu", "kernel": "trace Merkle tree (Poseidon2 leaf hash + levels)",
                              "achieved": valu_achieved, "unit": "M perm/s",
                              "peak": peak["mperm_per_s"] if peak else None,
                              "frac": valu_achieved / peak["mperm_per_s"] if peak else None,
                              "frac_at_measured_clock": (valu_achieved / peak["mperm_per_s_at_measured_clock"]
                                                         if peak else None),
                              "impl_mad_floor": {
                                  "mads_per_perm": peak["impl_mads_per_perm"] if peak else None,
                                  "mperm_per_s": peak["impl_mad_floor_mperm_per_s"] if peak else None,
                                  "frac": (valu_achieved / peak["impl_mad_floor_mperm_per_s"]
                                           if peak and peak["impl_mad_floor_mperm_per_s"] else None),
                                  "frac_at_measured_clock": (
                                      valu_achieved / peak["impl_mad_floor_mperm_per_s_at_measured_clock"]
                                      if peak and peak["impl_mad_floor_mperm_per_s_at_measured_clock"] else None),
                                  "note": "the shipped multiplier's own MAD count (9 x 29-bit limbs, carry-free "
                                          "columns) at the same MAD rate: the kernel's distance from its "
                                          "instruction floor; the 128-MAD peak above is the 8 x 32-bit floor, whose "
                                          "carry chains cost more than the extra MADs (DESIGN.md)"},
                              "peak_source": peak["source"] if peak else "profiles/r02_rates.json missing",
                              "fr_mul_achieved_g_per_s": valu_achieved * FR_MUL_PER_PERM / 1e3,
                              "fr_mul_peak_g_per_s": peak["gfrmul_per_s"] if peak else None,
                              "register_resident_chain_mperm_per_s": ctx.calibrate_poseidon2(),
                              "register_resident_chain_note": "k_calib_perm: dependent permutation chains in "
                                                              "registers, a latency-bound probe and not a peak "
                                                              "(the tree's leaf kernel outruns it)",
                              "valu_issue": valu_issue(["k_hash_rows1<11u, 1>", "k_merkle_level<11u, 1>"]),
                              "valu_issue_source": VALU_SRC.get("src"),
                              "perms": trace_perms, "fr_mul_per_perm": FR_MUL_PER_PERM, "ms": merkle_ms},
        }
        out["box_speed"] = box_speed(ctx, sclk, clocks.status, ms_per_step)
        if table is not None:
            out.update(table)
        if shard and world > 1:
            out["exchange"] = ctx.exchange_plan(h, w, q)
        if world == 1 and not shard and args.inflight > 1:
            out["inflight"] = inflight(args, cfg, air, pub, trace, ctx, dtrace)
        if world == 1 and not shard and not args.no_host_trace_leg:
            out["prove_time_host_trace_s"] = host_trace_leg(args, ctx, trace, air, pub)
            out["rows_per_s_host_trace"] = h / out["prove_time_host_trace_s"]["median"]
            if args.inflight > 1:
                out["inflight_host_trace"] = inflight(args, cfg, air, pub, trace, ctx, dtrace, host=True)
    ctx.dev_free(dtrace)
    return out, ctx


def air_log_q(air, cfg) -> int:
    import ctypes
    from linea_stark_prover_amd import _lib
    desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
    lq = ctypes.c_uint32()
    _lib.check(_lib.lib().lsp_log_quotient_degree(desc, len(desc), cfg.public_degree, ctypes.byref(lq)))
    return lq.value


def host_trace_leg(args, ctx, trace, air, pub):
    """SURVEY 8(d) rows/s: wall time including the H2D of the trace (pageable
    host array -> HBM inside lsp_prove), K steps after W warmups."""
    for _ in range(max(args.warmup, 1)):
        ctx.prove(trace, air, pub)
    ts = []
    for _ in range(max(args.steps, 1)):
        t = time.perf_counter()
        ctx.prove(trace, air, pub)
        ts.append(time.perf_counter() - t)
    return {"mean": sum(ts) / len(ts), "median": statistics.median(ts), "steps": len(ts),
            "trace_bytes": int(trace.nbytes),
            "note": "the trace starts in pageable host memory each step; value above starts with it in HBM"}


def batch_leg(args, dist, ctx, sizes):
    """BASELINE configs[4] (and configs[1] at N = 1): every rank proves its own
    independent 2^log_n trace (device-generated, rank-seeded), no data-path
    collective; value = all rows / the slowest rank's time (weak scaling)."""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import StarkConfig
    from linea_stark_prover_amd.replicas import rank_seed, timed_steps
    import numpy as np
    cfg = StarkConfig(seed=args.seed)
    a, d, _ = cfg.seeded()
    pub = np.concatenate([a, d])
    air = permutation_air(args.ncols)
    w = 2 * args.ncols + 2
    runs = []
    for log_n in sizes:
        h = 1 << log_n
        dtrace = ctx.gen_permutation_trace_device(log_n, args.ncols, a, d, seed=rank_seed(args.seed, dist.rank))
        step = lambda: ctx.prove(dtrace, air, pub, h, w)  # noqa: E731
        elapsed, proof = timed_steps(step, args.batch_leg_steps, 1, dist, sync=ctx.synchronize)
        ctx.dev_free(dtrace)
        if args.dump_batch_proofs:
            with open(f"{args.dump_batch_proofs}.{dist.rank}.{log_n}.bin", "wb") as f:
                f.write(proof)
        ok = bool(ctx.verify(proof, air, pub))  # every rank checks its own proof
        nok = int(round(dist.sum(1.0 if ok else 0.0)))
        run = {"log_n": log_n, "rows_per_rank": h, "steps": args.batch_leg_steps, "warmup": 1,
               "prove_time_s": elapsed / args.batch_leg_steps,
               "value": dist.world * h * args.batch_leg_steps / elapsed, "unit": "trace-rows/s",
               "scaling": "weak",
               "workload": f"{args.ncols}x{args.ncols} permutation AIR, one independent 2^{log_n}-row proof per "
                           f"rank ({dist.world} rank(s))"}
        run["verified"] = nok == dist.world
        run["verified_ranks"] = nok
        runs.append(run)
    return {"runs": runs}


def wide_leg(args, dist, ctx, log_n):
    """BASELINE configs[2]: the synthetic wide AIR -- 4 LogUp
    lookups (3-column A, two 3-column tables) + 8 permutation groups of 6+6,
    W = 184, trace/src/lookup.rs:46-176 and air/src/lib.rs:57-114 -- standing in
    for zkevm.bin (.MISSING_LARGE_BLOBS:1), at 2^log_n rows, trace resident in
    HBM: one warm-up, then the median of --wide-steps proofs.  The trace is the
    one tests/test_gpu_fullsize_oracle.py checks (lsp_gen_wide_trace, host);
    what bounds the proof is read off phases_ms and the kernels' stamped VALU
    issue (k_quotient: "quotient-eval bound" in BASELINE's words)."""
    from linea_stark_prover_amd.prover import StarkConfig, gen_wide_trace
    from linea_stark_prover_amd.replicas import timed_steps
    import numpy as np
    cfg = StarkConfig(seed=args.seed)
    a, d, _ = cfg.seeded()
    pub = np.concatenate([a, d])
    t0 = time.perf_counter()
    trace, air = gen_wide_trace(log_n, a, d, seed=args.seed)
    gen_s = time.perf_counter() - t0
    h, w = trace.shape[0], trace.shape[1]
    dtrace = ctx.dev_alloc(trace.nbytes)
    step_s = []
    try:
        ctx.h2d(dtrace, trace)
        del trace
        step = lambda: ctx.prove(dtrace, air, pub, h, w)  # noqa: E731
        elapsed, proof = timed_steps(step, args.wide_steps, 1, dist, sync=ctx.synchronize, step_times=step_s)
        ctx.set_phase_timing(True)  # the phase breakdown from one more, untimed proof
        step()
        phases = {k: round(v, 3) for k, v in ctx.last_timings()}
        ctx.set_phase_timing(True, only=ROOFLINE_PHASES)
        verified = bool(ctx.verify(proof, air, pub))
    finally:
        ctx.dev_free(dtrace)
    q = 1 << air_log_q(air, cfg)
    N = h << cfg.log_blowup
    med = statistics.median(step_s)
    leaf_perms = N * ((w + 1) // 2)  # the trace tree's leaves: ceil(w/2) permutations per LDE row
    merkle_ms = phases.get("merkle tree")
    out = {"workload": f"wide AIR (4 LogUp lookups + 8 permutation groups of 6+6), 2^{log_n} rows (w={w}, q={q})",
           "stands_in_for": "BASELINE configs[2]: Linea zkEVM trace from zkevm.bin, 2^20 rows (absent: "
                            ".MISSING_LARGE_BLOBS:1)",
           "steps": args.wide_steps, "warmup": 1, "prove_time_median_s": med, "prove_time_s": elapsed / args.wide_steps,
           "value": h / med, "unit": "trace-rows/s", "verified": verified, "phases_ms": phases,
           "trace_gen_s_host": round(gen_s, 2),
           "trace_tree_mperm_per_s": (leaf_perms + N - 1) / (merkle_ms * 1e-3) / 1e6 if merkle_ms else None,
           "valu_issue_k_quotient": valu_issue(["k_quotient"], "_wide"),
           "valu_issue_leaf_hash": valu_issue(["k_hash_rows"], "_wide"),
           "valu_issue_source": VALU_SRC.get("_wide")}
    return out


def shape_leg(args, dist, ctx, ncols):
    """The shape of the reference's only measured run (bench.log:1-20: a
    permutation over 6 'from' + 6 'to' columns, w = 14, 2^19 rows, 8 quotient
    chunks; 342 s on its CPU, bench.log:18), same K/W as the main leg, trace
    resident in HBM (device-generated)."""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import StarkConfig
    from linea_stark_prover_amd.replicas import timed_steps
    import numpy as np
    cfg = StarkConfig(seed=args.seed)
    a, d, _ = cfg.seeded()
    pub = np.concatenate([a, d])
    air = permutation_air(ncols)
    w, h = 2 * ncols + 2, 1 << args.log_n
    dtrace = ctx.gen_permutation_trace_device(args.log_n, ncols, a, d, seed=args.seed)
    step_s = []
    try:
        step = lambda: ctx.prove(dtrace, air, pub, h, w)  # noqa: E731
        elapsed, proof = timed_steps(step, args.steps, max(args.warmup, 1), dist, sync=ctx.synchronize,
                                     step_times=step_s)
        ctx.set_phase_timing(True)  # the phase breakdown from one more, untimed proof
        step()
        phases = {k: round(v, 3) for k, v in ctx.last_timings()}
        ctx.set_phase_timing(True, only=ROOFLINE_PHASES)
    finally:
        ctx.dev_free(dtrace)
    t = elapsed / args.steps
    out = {"workload": f"{ncols}x{ncols} permutation AIR, 2^{args.log_n} rows (w={w}, q="
                       f"{1 << air_log_q(air, cfg)}): the shape of bench.log:18-20",
           "steps": args.steps, "warmup": max(args.warmup, 1), "prove_time_s": t,
           "prove_time_median_s": statistics.median(step_s) if step_s else None,
           "value": h / t, "unit": "trace-rows/s", "verified": bool(ctx.verify(proof, air, pub)),
           "phases_ms": phases, "proof_of_work_bits": cfg.proof_of_work_bits,
           "reference_s": 342.0, "reference_source": "bench.log:18 (6+6 columns, w = 14, 2^19 rows, CPU)",
           "speedup_vs_reference": 342.0 / t if args.log_n == 19 else None}
    if args.shape_pow_bits > 0:
        try:
            out["with_pow"] = shape_pow_leg(args, dist, ctx, ncols, args.shape_pow_bits)
        except Exception as e:  # the leg above is still reported
            out["with_pow"] = {"error": f"{type(e).__name__}: {e}"}
    return out


def shape_pow_leg(args, dist, ctx, ncols, bits):
    """bench.log's run ground a proof-of-work witness (bench.log:65: 19.3 s of its
    342 s), which bin/src/main.rs:62 now sets to 0 bits with the comment //29: the
    same shape with `bits` bits on a context of its own (the grind is part of
    every timed proof; the witness is fixed by the transcript, so every step does
    the same work).  1 warm-up + 2 timed proofs."""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig
    from linea_stark_prover_amd.replicas import timed_steps
    import numpy as np
    cfg = StarkConfig(seed=args.seed, proof_of_work_bits=bits)
    a, d, _ = cfg.seeded()
    pub = np.concatenate([a, d])
    air = permutation_air(ncols)
    w, h = 2 * ncols + 2, 1 << args.log_n
    c = Context(cfg, device=ctx.device)
    try:
        dtrace = c.gen_permutation_trace_device(args.log_n, ncols, a, d, seed=args.seed)
        try:
            step = lambda: c.prove(dtrace, air, pub, h, w)  # noqa: E731
            elapsed, proof = timed_steps(step, 2, 1, dist, sync=c.synchronize)
            phases = dict(c.last_timings())
        finally:
            c.dev_free(dtrace)
        t = elapsed / 2
        grind_ms = phases.get("grind for proof-of-work witness", float("nan"))
        witness = pow_witness(proof)
        # the device grinds 2^22 candidates per launch (prove.cpp grind_device),
        # smallest first: the candidates this proof tested, their rate, and the
        # expected cost at `bits` (2^bits candidates) -- one proof's grind_ms is
        # one draw of a geometric witness, not the cost
        batch = 1 << 22
        tested = (witness // batch + 1) * batch
        rate = tested / (grind_ms * 1e-3) if grind_ms == grind_ms and grind_ms > 0 else None
        return {"proof_of_work_bits": bits, "steps": 2, "warmup": 1, "prove_time_s": t,
                "grind_ms": round(grind_ms, 3), "witness": witness, "candidates_tested": tested,
                "candidates_per_s": rate,
                "expected_grind_ms": (2 ** bits) / rate * 1e3 if rate else None,
                "expected_prove_time_s": t - grind_ms * 1e-3 + (2 ** bits) / rate if rate else None,
                "verified": bool(c.verify(proof, air, pub)),
                "reference_s": 342.0, "reference_grind_s": 19.3,
                "speedup_vs_reference": 342.0 / t if args.log_n == 19 else None,
                "note": "the grind is one Poseidon2 permutation per candidate witness (k_grind), "
                        "smallest witness first, as HashChallenger::grind"}
    finally:
        c.close()


def pow_witness(proof: bytes) -> int:
    """the proof-of-work witness of a serialized proof (csrc/proof.cpp layout:
    header, 2 roots, 2w + q opened values, FRI roots, final polynomial, then
    the witness, canonical little-endian)"""
    import struct
    _log_h, log_q, w, _nq, nr, nf = struct.unpack_from("<6I", proof, 8)
    off = 8 + 24 + 32 * (2 + 2 * w + (1 << log_q) + nr + nf)
    return int.from_bytes(proof[off:off + 32], "little")


def shard_leg_sizes(args, world):
    if args.shard_leg == "none" or args.shard or args.air != "perm":
        return []
    if args.shard_leg == "auto":
        return [24] + ([26] if world == 8 else [])
    return [int(x) for x in args.shard_leg.split(",") if x]


WATCHDOG_EXIT = 3  # exit status of every rank whose sharded leg hung


def guarded_shard_leg(args, dist, ctx, sizes, out, leg=None):
    """Run the C4 leg under a per-rank watchdog: if any collective hangs, rank
    0 still prints the main line (with the failure noted) and every rank exits
    with WATCHDOG_EXIT, so the run's status reports the hang
    (tests/test_replicas.py simulates one)."""
    done = threading.Event()
    leg = leg or shard_leg

    def watchdog():
        if done.wait(args.shard_timeout):
            return
        if dist.rank == 0 and out is not None:
            out["sharded"] = {"error": f"sharded leg exceeded {args.shard_timeout:.0f} s on rank 0; abandoned"}
            print(json.dumps(out), flush=True)
        sys.stdout.flush()
        os._exit(WATCHDOG_EXIT)

    threading.Thread(target=watchdog, daemon=True).start()
    try:
        return leg(args, dist, ctx, sizes)
    except Exception as e:  # the main line is still reported
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        done.set()


def shard_leg(args, dist, ctx, sizes):
    """one proof per size sharded over every rank."""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.replicas import timed_steps
    from linea_stark_prover_amd.prover import StarkConfig
    import ctypes
    import numpy as np
    from linea_stark_prover_amd import _lib

    world, rank = dist.world, dist.rank
    cfg = StarkConfig(seed=args.seed)
    a, d, _ = cfg.seeded()
    pub = np.concatenate([a, d])
    air = permutation_air(args.ncols)
    w = 2 * args.ncols + 2
    comm = "solo"
    if world > 1:
        from linea_stark_prover_amd import shard as S
        ndev = ctypes.c_int()
        _lib.check(_lib.lib().lsp_device_count(ctypes.byref(ndev)))
        comm = args.shard_comm
        if comm == "auto":
            local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
            comm = "rccl" if ndev.value >= local_world and args.device is None else "gloo"
        if comm == "rccl":
            S.attach_rccl(ctx)
        else:
            S.GlooComm().attach(ctx)
        seen = ctx.comm_info()[1]  # after the attach's allgather/bcast self-test
    else:
        seen = 1
    res = {"comm": comm, "n_ranks_seen": seen, "scaling": "strong", "host_threads": ctx.host_threads(), "runs": []}
    for log_n in sizes:
        h = 1 << log_n
        dtrace = ctx.gen_permutation_trace_device(log_n, args.ncols, a, d, seed=args.seed)
        if world > 1:
            from linea_stark_prover_amd import shard as S
            step = lambda: S.prove_sharded(ctx, dtrace, air, pub, h, w)  # noqa: E731
        else:
            step = lambda: ctx.prove(dtrace, air, pub, h, w)  # noqa: E731
        elapsed, proof = timed_steps(step, args.shard_leg_steps, args.shard_leg_warmup, dist,
                                     sync=ctx.synchronize)
        ctx.dev_free(dtrace)
        table = collective_table(ctx, dist) if world > 1 else None
        run = {"log_n": log_n, "rows": h, "steps": args.shard_leg_steps, "warmup": args.shard_leg_warmup,
               "prove_time_s": elapsed / args.shard_leg_steps,
               "value": h * args.shard_leg_steps / elapsed, "unit": "trace-rows/s",
               "workload": f"{args.ncols}x{args.ncols} permutation AIR, 2^{log_n} rows, one proof over {world} "
                           f"rank(s)", "proof_bytes": len(proof) if proof else 0}
        if table is not None:
            run.update(table)
        if world > 1:  # the inverse-NTT exchange this proof chose, on the attach-time calibration
            run["exchange"] = ctx.exchange_plan(h, w, 1 << air_log_q(air, cfg))
        if rank == 0:
            t = time.perf_counter()
            run["verified"] = bool(ctx.verify(proof, air, pub))
            run["verify_s"] = time.perf_counter() - t
        res["runs"].append(run)
    if world > 1:
        from linea_stark_prover_amd import shard as S
        S.detach(ctx)
    return res


def collective_table(ctx, dist):
    """The last sharded proof's collectives on every rank (lsp_comm_log): one
    row per collective in issue order -- op, bytes per rank, root, what it
    carried, and each rank's device ms around it (the wait for the slowest
    peer included) -- plus each rank's communicator creation time, so an
    8-GPU run's curve can be read exchange by exchange.  `schedule_identical`
    checks what RCCL needs: every rank issued the same (op, bytes, root)
    sequence."""
    log, init_ms = ctx.comm_log()
    logs = dist.all_gather_object((log, init_ms))
    ref = [(e["op"], e["bytes"], e["root"]) for e in logs[0][0]]
    same = all([(e["op"], e["bytes"], e["root"]) for e in lg] == ref for lg, _ in logs)
    rows = []
    for i, e in enumerate(logs[0][0]):
        rows.append({"op": e["op"], "bytes": e["bytes"], "root": e["root"], "tag": e["tag"],
                     "ms_by_rank": [round(lg[i]["ms"], 3) if i < len(lg) else None for lg, _ in logs]})
    by_tag = {}
    for r in rows:
        t = by_tag.setdefault(r["tag"], {"count": 0, "bytes": 0, "max_rank_ms": 0.0})
        t["count"] += 1
        t["bytes"] += r["bytes"]
        t["max_rank_ms"] = round(t["max_rank_ms"] + max(x for x in r["ms_by_rank"] if x is not None), 3)
    return {"collectives": rows, "collectives_by_tag": by_tag, "schedule_identical": same,
            "comm_init_ms_by_rank": [round(i, 3) for _, i in logs]}


def inflight(args, cfg, air, pub, trace, ctx, dtrace, host=False):
    """Production throughput mode: P independent proofs in flight on one GPU
    (P contexts = P HIP streams, one host thread each), so one proof's
    latency-bound phases (narrow Merkle levels, transcript, tree tops) overlap
    another's hashing.  host=True: every proof starts from the trace in host
    memory (the drop-in prove(RowMajorMatrix)), so one context's PCIe upload
    overlaps the others' compute instead of preceding its own proof.
    Reported beside `value` (the sequential single-proof rate), never instead
    of it."""
    from linea_stark_prover_amd.prover import Context
    P, K = args.inflight, max(args.steps, 2)
    h, w = trace.shape[0], trace.shape[1]
    ctxs, ptrs = [ctx], [dtrace]
    for _ in range(P - 1):
        c = Context(cfg, device=ctx.device)
        c.set_phase_timing(True, only=ROOFLINE_PHASES)
        if host:
            p = None
            c.prove(trace, air, pub)  # warm
        else:
            p = c.dev_alloc(trace.nbytes)
            c.h2d(p, trace)
            c.prove(p, air, pub, h, w)  # warm
        ctxs.append(c)
        ptrs.append(p)
    for c in ctxs:
        c.synchronize()

    def worker(i):
        for _ in range(K):
            if host:
                ctxs[i].prove(trace, air, pub)
            else:
                ctxs[i].prove(ptrs[i], air, pub, h, w)

    t = time.perf_counter()
    th = [threading.Thread(target=worker, args=(i,)) for i in range(P)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t
    for c, p in zip(ctxs[1:], ptrs[1:]):
        if p is not None:
            c.dev_free(p)
        c.close()
    return {"proofs_in_flight": P, "proofs": P * K, "value": P * K * h / dt, "unit": "trace-rows/s",
            "ms_per_proof": dt / (P * K) * 1e3,
            "note": ("independent proofs on P streams of one GPU, each trace uploaded from pageable host memory "
                     "inside its proof" if host else "independent proofs on P streams of one GPU") +
                    "; value above is one proof at a time"}


NTT_MADS_PER_PRODUCT = 162  # the NTT's 29-bit-limb product: 81 limb products + 81 reduction MADs


def ntt_impl_floor(frmul_gps, peak):
    """The LDE's products against the shipped multiplier's own MAD count (as
    roofline_valu.impl_mad_floor does for Poseidon2): the kernel's distance from
    an instruction stream of nothing but its products' MADs."""
    if not peak:
        return None
    floor = peak["mad_per_s"] / NTT_MADS_PER_PRODUCT / 1e9
    clk = peak["mperm_per_s_at_measured_clock"] / peak["mperm_per_s"]
    return {"mads_per_product": NTT_MADS_PER_PRODUCT, "g_per_s": floor, "frac": frmul_gps / floor,
            "frac_at_measured_clock": frmul_gps / (floor * clk)}


def valu_peak():
    """Chip peak for Poseidon2 hashing from the committed instruction-rate
    probe: v_mad_u64_u32 at C cycles per wave64 per SIMD (profiles/
    r02_rates.json) -> SIMDS * 64 / C MADs per cycle; one Fr product = 128 MADs
    (8 x 32-bit limbs), one permutation = 230 products.  At the nominal 2.4 GHz
    and at the clock the probe's MAD loop held."""
    try:
        r = json.load(open(RATES_FILE))
    except (OSError, ValueError):
        return None
    cyc = r["peak_basis"]["v_mad_u64_u32_cycles"]
    ghz_meas = r["peak_basis"]["measured_ghz"]
    mads = SIMDS * 64 / cyc * NOMINAL_GHZ * 1e9
    perm = mads / (MAD_PER_FR_MUL * FR_MUL_PER_PERM)
    floor = impl_mads_per_perm()
    return {"mad_per_s": mads, "gfrmul_per_s": mads / MAD_PER_FR_MUL / 1e9, "mperm_per_s": perm / 1e6,
            "mperm_per_s_at_measured_clock": perm / 1e6 * ghz_meas / NOMINAL_GHZ,
            "impl_mads_per_perm": floor,
            "impl_mad_floor_mperm_per_s": mads / floor / 1e6 if floor else None,
            "impl_mad_floor_mperm_per_s_at_measured_clock":
                mads / floor / 1e6 * ghz_meas / NOMINAL_GHZ if floor else None,
            "source": f"profiles/r02_rates.json: v_mad_u64_u32 {cyc} cycles per wave64 per SIMD x {SIMDS} SIMDs "
                      f"at {NOMINAL_GHZ} GHz; {MAD_PER_FR_MUL} MADs per Fr product, {FR_MUL_PER_PERM} products "
                      f"per permutation (measured clock under MAD load {ghz_meas} GHz)"}


def impl_mads_per_perm():
    """v_mad_u64_u32 per permutation in the shipped multiplier, counted in the
    generated asm (csrc/fr29_mul_gfx950_blk.inc: f29_mul_asm / f29_sqr_asm):
    46 S-boxes x (3 squares + 2 products) for x^11 (rf = 8, rp = 22) -- the
    instruction floor of this representation (9 x 29-bit limbs: 81 + 72 + 9
    MADs per product, 45 + 72 + 9 per square), against which the kernel's
    non-MAD overhead is measured."""
    try:
        src = open(os.path.join(ROOT, "linea_stark_prover_amd", "csrc", "fr29_mul_gfx950_blk.inc")).read()
    except OSError:
        return None
    mul, sqr = src.split("f29_sqr_asm", 1) if "f29_sqr_asm" in src else (src, "")
    nm, ns = mul.count("v_mad_u64_u32"), sqr.count("v_mad_u64_u32")
    return (3 * 8 + 22) * (3 * ns + 2 * nm) if nm and ns else None


def valu_issue(kernels, kind=""):
    """Time-weighted VALU issue share of the named kernels from the committed
    PMC passes (tools/pmc_stamp.sh -> profiles/*_valu_pmc{kind}.json; kind
    "_wide": the wide-AIR proof's passes): SIMD cycles with a VALU instruction
    issuing (SQ_ACTIVE_INST_VALU over all waves) / (1024 SIMDs x kernel
    cycles).  Only a profile stamped with this library's source hash counts
    (lib_src_sha16); else None, with the reason in VALU_SRC[kind or "src"]."""
    import glob
    d, src, stale = None, None, []
    key = kind or "src"
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_valu_pmc{kind}.json"))):
        try:
            x = json.load(open(path))
        except (OSError, ValueError):
            continue
        if x.get("lib_src_sha16") == LIB_SRC:
            d, src = x, os.path.relpath(path, ROOT)
        else:
            stale.append(os.path.basename(path))
    if not d:
        VALU_SRC[key] = (f"null: no profiles/*_valu_pmc{kind}.json measured on this build (lib_src_sha16 {LIB_SRC}; "
                         f"{len(stale)} older profile(s) skipped)")
        return None
    VALU_SRC[key] = src
    ks = [v for k, v in d["kernels"].items() if any(k.startswith(p) for p in kernels)]
    ms = sum(v["ms"] for v in ks)
    return round(sum(v["valu_issue"] * v["ms"] for v in ks) / ms, 3) if ms else None


def lde_traffic(log_n, w):
    """HBM bytes per coset_lde_batch from the rocprofv3 PMC passes of
    tools/pmc_round.sh (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction), kept in
    profiles/; None when no measurement of this size was made on this build
    (lib_src_sha16), with the reason in TRAFFIC_SRC."""
    import glob
    best, stale = None, 0
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_lde_traffic.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("h") == (1 << log_n) and d.get("w") == w:
            if d.get("lib_src_sha16") == LIB_SRC:
                best = d["traffic_bytes"]
                TRAFFIC_SRC[(log_n, w)] = os.path.relpath(path, ROOT)
            else:
                stale += 1
    if best is None:
        TRAFFIC_SRC[(log_n, w)] = (f"null: no profiles/*_lde_traffic.json of 2^{log_n} x {w} measured on this build "
                                   f"(lib_src_sha16 {LIB_SRC}; {stale} older profile(s) skipped)")
    return best


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> int:
    """the host cores this process may use: the scheduler affinity, capped by the
    pool's per-GPU share (OMP_NUM_THREADS / nproc on the GPU box)"""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


def _cpu_prove_times(cref, args, log_n, runs, threads, warmup=0):
    """`warmup` untimed + `runs` timed full proofs of the C restatement at 2^log_n rows"""
    p = cref.setup(args.seed)
    tb, w = cref.gen_perm_trace(p, log_n, args.ncols, seed=args.seed)
    air = cref.perm_air(args.ncols)
    ts = []
    for k in range(runs + warmup):
        t = time.perf_counter()
        cref.prove(p, tb, 1 << log_n, w, air, nthreads=threads)
        dt = time.perf_counter() - t
        if k >= warmup:
            ts.append(dt)
        # progress on stderr: a 2^19 CPU proof takes tens of seconds
        print(f"[cpu_baseline] 2^{log_n} {'warm-up' if k < warmup else f'run {k - warmup + 1}/{runs}'}: {dt:.2f} s",
              file=sys.stderr, flush=True)
    return ts


def cpu_baseline(args):
    """The oracle's C restatement (test infrastructure, used here only as the
    reported baseline) proving the headline workload -- the same AIR, size,
    conventions and seed (the 2^19 input) -- on the host, one
    thread per core of this process's CPU share: one warm-up, then the median
    of --cpu-runs timed proofs.  A smaller sample (--cpu-small-log-n) is
    reported beside it under `small_sample`."""
    from oracle import cref
    cref.build()
    threads = cpu_share()
    log_n = args.cpu_log_n if args.cpu_log_n is not None else args.log_n
    runs = max(args.cpu_runs, 1)
    ts = _cpu_prove_times(cref, args, log_n, runs, threads, max(args.cpu_warmup, 0))
    dt = statistics.median(ts)
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip())
    except (OSError, ValueError):
        nproc = None
    out = {"value": (1 << log_n) / dt, "unit": "trace-rows/s", "cores": threads, "kind": "port",
           "seconds": dt, "seconds_runs": [round(x, 3) for x in ts], "warmup": max(args.cpu_warmup, 0),
           "log_n": log_n, "nproc": nproc,
           "machine_cpus": os.cpu_count(), "cpu_model": cpu_model(),
           "sample": f"oracle/lsp_oracle.c full prove of the headline workload: {args.ncols}x{args.ncols} "
                     f"permutation AIR at 2^{log_n} rows (same AIR, conventions and seed as the GPU line), "
                     f"median of {len(ts)} runs ({max(args.cpu_warmup, 0)} warm-up), {threads} threads = this "
                     f"process's CPU share "
                     f"(affinity / OMP_NUM_THREADS)",
           "gpu_speedup": None}
    if args.cpu_small_log_n and args.cpu_small_log_n < log_n:
        ts2 = _cpu_prove_times(cref, args, args.cpu_small_log_n, 3, threads)
        out["small_sample"] = {"log_n": args.cpu_small_log_n, "seconds": statistics.median(ts2),
                               "value": (1 << args.cpu_small_log_n) / statistics.median(ts2),
                               "seconds_runs": [round(x, 3) for x in ts2]}
    return out


if __name__ == "__main__":
    sys.exit(main())
