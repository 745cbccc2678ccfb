"""Same-process A/B of two builds of liblsp_hip.so: both libraries are loaded
side by side (distinct paths, RTLD_LOCAL), each with its own context and
device copy of the same 2^log_n trace, and proofs alternate A, B, A, B, ...
so both see the same clocks, the same box and the same host state.  Box-to-box
and process-to-process noise (about 1 ms at 2^19) does not enter the paired
differences; effects of 0.1 ms become visible.

    python tools/ab_inproc.py libA.so libB.so [--log-n 19] [--pairs 30] [--env-b VAR=VAL]

--env-b sets environment variables around B's proofs only (for switches the
library reads per call; the ones it caches at first use need two builds).
Prints per-library median / mean / min, the median of the paired differences
B - A and how often B won, and checks that A and B made the same proof.
"""
import argparse
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(path):
    from linea_stark_prover_amd import _lib
    L = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_NOW)
    for name, (res, args) in _lib._SIGS.items():
        f = getattr(L, name, None)  # an older build lacks the later entry points
        if f is None:
            continue
        f.restype = res
        f.argtypes = args
    return L


class LspParamsR3(ctypes.Structure):
    """lsp_params as round 3's library took it (no struct_size, no transcript
    switches): --r3-abi lets a round-3 build race the current one"""
    _fields_ = [("sbox_degree", ctypes.c_uint32), ("rounds_f", ctypes.c_uint32), ("rounds_p", ctypes.c_uint32),
                ("round_constants", ctypes.c_void_p), ("log_blowup", ctypes.c_uint32),
                ("log_final_poly_len", ctypes.c_uint32), ("num_queries", ctypes.c_uint32),
                ("proof_of_work_bits", ctypes.c_uint32), ("public_degree", ctypes.c_int32),
                ("internal_diag", ctypes.c_void_p), ("external_mds", ctypes.c_void_p)]


class Side:
    def __init__(self, path, log_n, ncols=3, r3_abi=False):
        import numpy as np
        from linea_stark_prover_amd import _lib
        from linea_stark_prover_amd.air import permutation_air
        from linea_stark_prover_amd.prover import StarkConfig
        self.name = os.path.basename(path)
        self.L = L = load(path)
        cfg = StarkConfig()
        a, d, rc = cfg.seeded()
        self.rc = rc
        self.pub = np.ascontiguousarray(np.concatenate([a, d]))
        P = LspParamsR3 if r3_abi else _lib.LspParams
        if r3_abi:  # this side's own CDLL: its create takes the older struct
            L.lsp_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(LspParamsR3), ctypes.POINTER(ctypes.c_void_p)]
        p = P(sbox_degree=cfg.sbox_degree, rounds_f=cfg.rounds_f, rounds_p=cfg.rounds_p,
                           round_constants=rc.ctypes.data, log_blowup=cfg.log_blowup,
                           log_final_poly_len=cfg.log_final_poly_len, num_queries=cfg.num_queries,
                           proof_of_work_bits=cfg.proof_of_work_bits, public_degree=cfg.public_degree)
        self.h = ctypes.c_void_p()
        self._chk(L.lsp_ctx_create(0, ctypes.byref(p), ctypes.byref(self.h)))
        self.rows, self.w = 1 << log_n, 2 * ncols + 2
        self.dtrace = ctypes.c_void_p()
        self._chk(L.lsp_dev_alloc(self.h, self.rows * self.w * 32, ctypes.byref(self.dtrace)))
        self._chk(L.lsp_gen_permutation_trace_device(self.h, 1, log_n, ncols, a.ctypes.data, d.ctypes.data,
                                                     self.dtrace))
        desc = permutation_air(ncols).descriptor()
        self.desc = (ctypes.c_int32 * len(desc))(*desc)

    def _chk(self, rc):
        if rc != 0:
            msg = self.L.lsp_last_error(self.h if hasattr(self, "h") else None)
            raise RuntimeError(f"{self.name}: lsp error {rc}: {msg.decode() if msg else ''}")

    def prove(self):
        """one proof, timed like bench.py's step (host to host), serialized"""
        self._chk(self.L.lsp_synchronize(self.h))
        t = time.perf_counter()
        pf = ctypes.c_void_p()
        self._chk(self.L.lsp_prove(self.h, self.dtrace, self.rows, self.w, self.desc, len(self.desc),
                                   self.pub.ctypes.data, 2, 1, ctypes.byref(pf)))
        n = ctypes.c_size_t()
        self._chk(self.L.lsp_proof_serialize(pf, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        self._chk(self.L.lsp_proof_serialize(pf, buf, n.value, ctypes.byref(n)))
        out = buf.raw[:n.value]
        self.L.lsp_proof_free(pf)
        return time.perf_counter() - t, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--log-n", type=int, default=19)
    ap.add_argument("--pairs", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--env-b", default=None, help="VAR=VAL[,VAR=VAL...] set around B's proofs only")
    ap.add_argument("--r3-abi", default="", help="a, b or ab: that side is a round-3 build (its lsp_params)")
    ap.add_argument("--swap", action="store_true",
                    help="one library + --env-b: apply the switch to context B, then to context A, half the pairs each")
    args = ap.parse_args()
    A, B = Side(args.a, args.log_n, r3_abi="a" in args.r3_abi), Side(args.b, args.log_n, r3_abi="b" in args.r3_abi)
    envs = [kv.split("=", 1) for kv in args.env_b.split(",")] if args.env_b else []
    if envs:
        B.name += f" [{args.env_b}]"

    def with_env(side):
        old = {k: os.environ.get(k) for k, _ in envs}
        for k, v in envs:
            os.environ[k] = v
        try:
            return side.prove()
        finally:
            for k, v in old.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v

    for _ in range(args.warmup):
        A.prove()
        with_env(B)
    ta, tb, diff = [], [], []
    same = True
    # Two contexts differ by themselves (buffer placement: +-0.3 ms per 2^19
    # proof in A/A runs).  With --swap and one library, the switch moves from
    # context B to context A halfway, so that bias cancels in the differences.
    swap = args.swap and args.a == args.b and envs
    for i in range(args.pairs):
        second = swap and i >= args.pairs // 2
        run_a = (lambda: with_env(A)) if second else A.prove
        run_b = B.prove if second else (lambda: with_env(B))
        # alternate which side goes first, so a drift within a pair cancels
        if i % 2 == 0:
            (x, pa), (y, pb) = run_a(), run_b()
        else:
            (y, pb), (x, pa) = run_b(), run_a()
        if second:
            x, y = y, x  # x: without the switch, y: with it
        ta.append(x)
        tb.append(y)
        diff.append(y - x)
        same = same and pa == pb
    ms = lambda v: v * 1e3  # noqa: E731
    for name, t in ((A.name, ta), (B.name, tb)):
        print(f"{name:28s} median {ms(statistics.median(t)):7.2f} ms  mean {ms(statistics.mean(t)):7.2f}  "
              f"min {ms(min(t)):7.2f}  ({len(t)} proofs, 2^{args.log_n})")
    wins = sum(1 for d in diff if d < 0)
    print(f"B - A: median {ms(statistics.median(diff)):+.3f} ms, mean {ms(statistics.mean(diff)):+.3f} ms; "
          f"B faster in {wins}/{len(diff)} pairs; identical proofs: {same}")


if __name__ == "__main__":
    main()
