"""Whole-proof parity at full size: the GPU proof of the 3x3 permutation AIR
against the C oracle's proof of the same seeded trace, byte for byte.

The oracle (oracle/lsp_oracle.c, test infrastructure) is only the checker; it
takes minutes at 2^22 on 16 host threads, which is why this is a tool run
recorded under profiles/ and not part of the GPU test suite.
Usage: python tools/full_oracle_proof.py LOG_N[xNCOLS] | wLOG_N ...   (e.g. 19 22 19x6 w20; NCOLS 3 by default;
       wLOG_N: the wide C3 AIR, 4 LogUp lookups + 8 groups of 6+6, W = 184;
       threads: LSP_ORACLE_THREADS, default 16)"""
import hashlib
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from linea_stark_prover_amd.air import permutation_air  # noqa: E402
from linea_stark_prover_amd.prover import Context, StarkConfig  # noqa: E402
from linea_stark_prover_amd.build import library_hash, source_hash  # noqa: E402
from oracle import cref  # noqa: E402

nthreads = int(os.environ.get("LSP_ORACLE_THREADS", "16"))
p = cref.setup()
pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
ok_all = True
print(f"lib_src_sha16={library_hash() or source_hash()} (the library these GPU proofs come from)", flush=True)


def heartbeat(stop):  # a line a minute while the oracle runs (long silent runs read as hung)
    t = time.time()
    while not stop.wait(60):
        print(f"  ... oracle running, {time.time() - t:.0f} s", flush=True)


with Context(StarkConfig(), device=0) as ctx:
    for arg in sys.argv[1:] or ["19"]:
        if arg.startswith("w"):  # the wide AIR
            from linea_stark_prover_amd.prover import gen_wide_trace
            log_n = int(arg[1:])
            a, d, _ = ctx.config.seeded()
            t0 = time.time()
            tr, air = gen_wide_trace(log_n, a, d)
            t1 = time.time()
            wpub = np.concatenate([a, d])
            gpu = ctx.prove(tr, air, wpub)
            t2 = time.time()
            stop = threading.Event()
            threading.Thread(target=heartbeat, args=(stop,), daemon=True).start()
            ref = cref.prove(p, tr.ctypes.data, 1 << log_n, tr.shape[1], air.descriptor(), nthreads=nthreads)
            stop.set()
            t3 = time.time()
            same = gpu == ref
            ok_all &= same
            print(f"log_n={log_n} wide AIR w={tr.shape[1]}: trace {t1 - t0:.1f} s; GPU proof {t2 - t1:.2f} s (incl. upload, "
                  f"first call); oracle proof {t3 - t2:.1f} s on {nthreads} threads; {len(gpu)} bytes; "
                  f"sha256 {hashlib.sha256(gpu).hexdigest()[:16]} / {hashlib.sha256(ref).hexdigest()[:16]}; "
                  f"byte-identical={same}; verified={ctx.verify(gpu, air, wpub)}", flush=True)
            del tr
            continue
        log_n, _, nc = arg.partition("x")
        log_n, ncols = int(log_n), int(nc or 3)
        t0 = time.time()
        tb, w = cref.gen_perm_trace(p, log_n, ncols)
        trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << log_n, w, 4)
        t1 = time.time()
        gpu = ctx.prove(trace, permutation_air(ncols), pub)
        t2 = time.time()
        stop = threading.Event()
        threading.Thread(target=heartbeat, args=(stop,), daemon=True).start()
        ref = cref.prove(p, tb, 1 << log_n, w, cref.perm_air(ncols), nthreads=nthreads)
        stop.set()
        t3 = time.time()
        same = gpu == ref
        ok_all &= same
        verified = ctx.verify(gpu, permutation_air(ncols), pub)
        print(f"log_n={log_n} {ncols}x{ncols} AIR w={w}: trace {t1 - t0:.1f} s; GPU proof {t2 - t1:.2f} s (incl. upload, first call); "
              f"oracle proof {t3 - t2:.1f} s on {nthreads} threads; {len(gpu)} bytes; "
              f"sha256 {hashlib.sha256(gpu).hexdigest()[:16]} / {hashlib.sha256(ref).hexdigest()[:16]}; "
              f"byte-identical={same}; verified={verified}", flush=True)
        del trace, tb
sys.exit(0 if ok_all else 1)
