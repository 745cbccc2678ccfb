"""Big-integer CPU restatement of the reference prover's hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker.  The product path (``linea_stark_prover_amd``) never calls it.

This is the *mini oracle*: plain Python integers, readable, slow (tiny sizes
only, log2(rows) <= ~8 for a full proof).  It restates

* the driver/AIR/trace crates of distributed-lab/linea-stark-prover
  (``air/src/lib.rs:57-167``, ``air/src/air_permutation.rs:21-23``,
  ``air/src/air_lookup.rs:37-39``, ``trace/src/permutation.rs:24-93``,
  ``trace/src/lookup.rs:46-176``, ``trace/src/lib.rs:94-106``,
  ``bin/src/config.rs:9-25``, ``bin/src/main.rs:29-96``), and
* the Plonky3 fork those crates call (distributed-lab/Plonky3 @ f888f90,
  pinned at ``Cargo.lock:505-711``; NOT present in this container).  The
  fork's algorithms are restated from upstream Plonky3 semantics of that era
  (``FieldAlgebra`` naming, Dec 2024 - Jan 2025), under the named conventions
  U1..U12 of SURVEY.md section 8(c).

Parity status: the reference ships no tests, fixtures or golden vectors and
its toolchain (cargo + the fork) is absent, so results that depend on the
fork's unpinned conventions (Poseidon2 constants/S-box/layers, transcript
order, sample_bits, grinding) are **parity unpinned**.  Results that are
mathematically unique (field constants, coset LDE values, selectors,
barycentric opened values, inverse denominators) are pinned by theorem and
cross-checked here by independent methods (naive polynomial evaluation).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------
# A1 -- BLS12-377 scalar field Fr (ark-bls12-377 0.5.0, Cargo.lock:51;
# used via p3-bls12-377-fr, bin/src/config.rs:1,9-10)
# ---------------------------------------------------------------------------
P = 0x12AB655E9A2CA55660B44D1E5C37B00159AA76FED00000010A11800000000001
TWO_ADICITY = 47
GENERATOR = 22  # U9: multiplicative generator (a quadratic non-residue)
ROOT_2_47 = pow(GENERATOR, (P - 1) >> TWO_ADICITY, P)
MONT_R = pow(2, 256, P)
MONT_R_INV = pow(MONT_R, P - 2, P)


def inv(x: int) -> int:
    x %= P
    if x == 0:
        raise ZeroDivisionError("inverse of zero in Fr")
    return pow(x, P - 2, P)


def two_adic_generator(bits: int) -> int:
    """p3-field TwoAdicField::two_adic_generator: root47^(2^(47-bits))."""
    assert 0 <= bits <= TWO_ADICITY
    return pow(ROOT_2_47, 1 << (TWO_ADICITY - bits), P)


def to_mont_bytes(x: int) -> bytes:
    """ark-ff in-memory form: Montgomery (R = 2^256), 4 x u64 little endian."""
    return ((x % P) * MONT_R % P).to_bytes(32, "little")


def from_mont_bytes(b: bytes) -> int:
    return int.from_bytes(b, "little") * MONT_R_INV % P


def to_canon_bytes(x: int) -> bytes:
    return (x % P).to_bytes(32, "little")


def from_be_bytes_mod_order(b: bytes) -> int:
    """ark-ff PrimeField::from_be_bytes_mod_order (trace/src/permutation.rs:102)."""
    return int.from_bytes(b, "big") % P


def bitrev(i: int, bits: int) -> int:
    out = 0
    for _ in range(bits):
        out = (out << 1) | (i & 1)
        i >>= 1
    return out


def reverse_slice_index_bits(v: list) -> list:
    n = len(v)
    bits = n.bit_length() - 1
    assert 1 << bits == n
    return [v[bitrev(i, bits)] for i in range(n)]


def log2_strict(n: int) -> int:
    b = n.bit_length() - 1
    assert n == 1 << b, f"{n} is not a power of two"
    return b


def log2_ceil(n: int) -> int:
    return 0 if n <= 1 else (n - 1).bit_length()


# ---------------------------------------------------------------------------
# U4/U5: the documented seeded generator that replaces thread_rng()
# (bin/src/main.rs:29-31,49).  SplitMix64; an Fr sample takes 4 words,
# masks to 253 bits and rejects values >= P.
# ---------------------------------------------------------------------------
MASK64 = (1 << 64) - 1
DEFAULT_SEED = 0x4C494E4541  # "LINEA"


class SplitMix64:
    def __init__(self, seed: int):
        self.state = seed & MASK64

    def next_u64(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def sample_fr(self) -> int:
        while True:
            v = 0
            for k in range(4):
                v |= self.next_u64() << (64 * k)
            v &= (1 << 253) - 1
            if v < P:
                return v

    def below(self, n: int) -> int:
        """Uniform integer in [0, n) (rejection on the top of 2^64)."""
        lim = (1 << 64) - ((1 << 64) % n)
        while True:
            x = self.next_u64()
            if x < lim:
                return x % n


# ---------------------------------------------------------------------------
# A3 -- Poseidon2Bls12337<3> (bin/src/config.rs:11), Perm::new_from_rng(8, 22)
# (bin/src/main.rs:49).  U1: S-box x^11.  U2: internal layer M_I = J + diag(d),
# s_i <- (s0 + s1 + s2) + d_i s_i, default d = (1, 1, 2) (the Bn254 template of
# upstream Plonky3's width-3 internal layer).  U3: external layer M_E, applied
# once before the first full round and after every full round, default
# circ(2, 1, 1) (s_i += s0 + s1 + s2).  Both are parameters (int_diag,
# ext_mds; None = default) so a caller whose fork uses other layers can set them.
# ---------------------------------------------------------------------------
DEFAULT_INT_DIAG = (1, 1, 2)
DEFAULT_EXT_MDS = (2, 1, 1, 1, 2, 1, 1, 1, 2)


@dataclass
class Poseidon2Params:
    sbox_degree: int = 11
    rounds_f: int = 8
    rounds_p: int = 22
    ext_initial: List[List[int]] = field(default_factory=list)   # rounds_f/2 x 3
    ext_terminal: List[List[int]] = field(default_factory=list)  # rounds_f/2 x 3
    internal: List[int] = field(default_factory=list)            # rounds_p
    int_diag: Optional[Sequence[int]] = None   # U2: d (3 ints mod P); None = (1, 1, 2)
    ext_mds: Optional[Sequence[int]] = None    # U3: M_E row-major (9 ints mod P); None = circ(2, 1, 1)


@dataclass
class Setup:
    alpha: int
    delta: int
    perm: Poseidon2Params


def setup_from_seed(seed: int = DEFAULT_SEED, sbox_degree: int = 11,
                    rounds_f: int = 8, rounds_p: int = 22) -> Setup:
    """Draw order mirrors bin/src/main.rs: alpha, delta (:30-31) then the
    Poseidon2 constants (:49) in Plonky3's new_from_rng order: initial
    external rounds, terminal external rounds, internal rounds."""
    rng = SplitMix64(seed)
    alpha = rng.sample_fr()
    delta = rng.sample_fr()
    half = rounds_f // 2
    ini = [[rng.sample_fr() for _ in range(3)] for _ in range(half)]
    ter = [[rng.sample_fr() for _ in range(3)] for _ in range(half)]
    internal = [rng.sample_fr() for _ in range(rounds_p)]
    return Setup(alpha, delta, Poseidon2Params(sbox_degree, rounds_f, rounds_p, ini, ter, internal))


def _ext_layer(s, m=None):
    """s <- M_E s; M_E = circ(2, 1, 1) (s_i += s0 + s1 + s2) unless given."""
    if m is None:
        t = (s[0] + s[1] + s[2]) % P
        return [(s[0] + t) % P, (s[1] + t) % P, (s[2] + t) % P]
    return [(m[3 * i] * s[0] + m[3 * i + 1] * s[1] + m[3 * i + 2] * s[2]) % P for i in range(3)]


def _int_layer(s, d=None):
    """s_i <- (s0 + s1 + s2) + d_i s_i; d = (1, 1, 2) unless given."""
    d = DEFAULT_INT_DIAG if d is None else d
    t = (s[0] + s[1] + s[2]) % P
    return [(t + d[i] * s[i]) % P for i in range(3)]


def permute(state: Sequence[int], pp: Poseidon2Params) -> List[int]:
    d = pp.sbox_degree
    m, dg = pp.ext_mds, pp.int_diag
    s = _ext_layer(list(state), m)
    for rc in pp.ext_initial:
        s = [pow((s[i] + rc[i]) % P, d, P) for i in range(3)]
        s = _ext_layer(s, m)
    for rc in pp.internal:
        s[0] = pow((s[0] + rc) % P, d, P)
        s = _int_layer(s, dg)
    for rc in pp.ext_terminal:
        s = [pow((s[i] + rc[i]) % P, d, P) for i in range(3)]
        s = _ext_layer(s, m)
    return s


PERM_COUNTER = [0]


def hash_iter(elems: Sequence[int], pp: Poseidon2Params) -> int:
    """A4 -- PaddingFreeSponge<Perm, 3, 2, 1> (bin/src/config.rs:12):
    overwrite-mode absorb of 2 elements per permutation, no padding, a final
    partial block only overwrites the lanes it has, output lane 0."""
    state = [0, 0, 0]
    it = list(elems)
    pos = 0
    while True:
        for i in range(2):
            if pos < len(it):
                state[i] = it[pos] % P
                pos += 1
            else:
                if i != 0:
                    PERM_COUNTER[0] += 1
                    state = permute(state, pp)
                return state[0]
        PERM_COUNTER[0] += 1
        state = permute(state, pp)


def compress(left: int, right: int, pp: Poseidon2Params) -> int:
    """A5 -- CompressionFunctionFromHasher<Hash, 2, 1> (bin/src/config.rs:17)."""
    return hash_iter([left, right], pp)


# ---------------------------------------------------------------------------
# A6/A7 -- MerkleTreeMmcs<Val, Val, Hash, Compress, 1> (bin/src/config.rs:19-20)
# Only equal-height matrices occur on this path (all commits here are of one
# height), which is the case restated.
# ---------------------------------------------------------------------------
@dataclass
class MerkleTree:
    mats: List[List[List[int]]]      # list of matrices, each a list of rows
    layers: List[List[int]]          # layers[0] = leaf digests ... [-1] = [root]

    @property
    def root(self) -> int:
        return self.layers[-1][0]

    @property
    def height(self) -> int:
        return len(self.mats[0])


def merkle_commit(mats: List[List[List[int]]], pp: Poseidon2Params) -> MerkleTree:
    h = len(mats[0])
    assert all(len(m) == h for m in mats), "equal heights only on this path"
    log2_strict(h)
    leaves = [hash_iter([x for m in mats for x in m[i]], pp) for i in range(h)]
    layers = [leaves]
    while len(layers[-1]) > 1:
        prev = layers[-1]
        layers.append([compress(prev[2 * i], prev[2 * i + 1], pp) for i in range(len(prev) // 2)])
    return MerkleTree(mats, layers)


def merkle_open(tree: MerkleTree, index: int) -> Tuple[List[List[int]], List[int]]:
    rows = [list(m[index]) for m in tree.mats]
    path = [tree.layers[i][(index >> i) ^ 1] for i in range(len(tree.layers) - 1)]
    return rows, path


def merkle_verify(root: int, index: int, rows: List[List[int]], path: List[int],
                  pp: Poseidon2Params) -> bool:
    cur = hash_iter([x for r in rows for x in r], pp)
    for i, sib in enumerate(path):
        if (index >> i) & 1:
            cur = compress(sib, cur, pp)
        else:
            cur = compress(cur, sib, pp)
    return cur == root


# ---------------------------------------------------------------------------
# A2 -- coset LDE (p3-dft Radix2DitParallel::coset_lde_batch, bin/src/config.rs:22)
# ---------------------------------------------------------------------------
def ntt(vals: List[int], root: int) -> List[int]:
    """Natural-order DFT: out[k] = sum_j vals[j] root^(jk)."""
    n = len(vals)
    if n == 1:
        return [vals[0] % P]
    even = ntt(vals[0::2], root * root % P)
    odd = ntt(vals[1::2], root * root % P)
    out = [0] * n
    w = 1
    for k in range(n // 2):
        t = w * odd[k] % P
        out[k] = (even[k] + t) % P
        out[k + n // 2] = (even[k] - t) % P
        w = w * root % P
    return out


def idft(vals: List[int]) -> List[int]:
    n = len(vals)
    root = inv(two_adic_generator(log2_strict(n)))
    ninv = inv(n)
    return [x * ninv % P for x in ntt(vals, root)]


def coset_lde_column(col: List[int], added_bits: int, shift: int) -> List[int]:
    """Values of the interpolant of ``col`` (on H_h) at shift * w_N^bitrev(i)."""
    h = len(col)
    coeffs = idft(col) + [0] * (h * ((1 << added_bits) - 1))
    big = len(coeffs)
    s = 1
    for i in range(big):
        coeffs[i] = coeffs[i] * s % P
        s = s * shift % P
    evals = ntt(coeffs, two_adic_generator(log2_strict(big)))
    return reverse_slice_index_bits(evals)


def coset_lde_batch(rows: List[List[int]], added_bits: int, shift) -> List[List[int]]:
    """Row-major h x w in, row-major bit-reversed N x w out.  ``shift`` may be
    one element (all columns) or a per-column list (batched quotient chunks)."""
    w = len(rows[0])
    shifts = shift if isinstance(shift, (list, tuple)) else [shift] * w
    cols = [coset_lde_column([r[c] for r in rows], added_bits, shifts[c]) for c in range(w)]
    return [[cols[c][i] for c in range(w)] for i in range(len(cols[0]))]


def eval_poly(coeffs: List[int], x: int) -> int:
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % P
    return acc


# ---------------------------------------------------------------------------
# A16/A17 -- HashChallenger<Val, Hash, 1> (bin/src/config.rs:23) + U8
# ---------------------------------------------------------------------------
class HashChallenger:
    def __init__(self, pp: Poseidon2Params, initial=None, mont_bits: bool = False):
        self.pp = pp
        self.input_buffer = list(initial or [])
        self.output_buffer: List[int] = []
        self.mont_bits = mont_bits  # U8 switch: sample_bits from the Montgomery form x * 2^256 mod r

    def observe(self, x: int):
        self.output_buffer.clear()
        self.input_buffer.append(x % P)

    def observe_slice(self, xs):
        for x in xs:
            self.observe(x)

    def _flush(self):
        out = hash_iter(self.input_buffer, self.pp)
        self.input_buffer = [out]
        self.output_buffer = [out]

    def sample(self) -> int:
        if not self.output_buffer:
            self._flush()
        return self.output_buffer.pop()

    def sample_bits(self, bits: int) -> int:
        x = self.sample()
        if self.mont_bits:
            x = x * MONT_R % P
        return x & ((1 << bits) - 1)

    def check_witness(self, bits: int, witness: int) -> bool:
        self.observe(witness)
        return self.sample_bits(bits) == 0

    def grind(self, bits: int) -> int:
        w = 0
        while True:
            probe = HashChallenger(self.pp, mont_bits=self.mont_bits)
            probe.input_buffer = list(self.input_buffer)
            probe.output_buffer = list(self.output_buffer)
            if probe.check_witness(bits, w):
                break
            w += 1
        assert self.check_witness(bits, w)
        return w


# ---------------------------------------------------------------------------
# AIR configs (air/src/air_permutation.rs, air/src/air_lookup.rs) and the
# constraint program of LineaAIR::eval (air/src/lib.rs:47-167)
# ---------------------------------------------------------------------------
@dataclass
class PermCfg:
    a_cols: List[int]
    b_cols: List[int]
    b_inv: int
    check: int

    def width(self):
        return len(self.a_cols) + len(self.b_cols) + 2


@dataclass
class LookupCfg:
    a_cols: List[int]
    b_cols: List[List[int]]
    a_filter: int
    b_filter: List[int]
    a_inv: int
    b_inv: List[int]
    occ: List[int]
    check: int

    def width(self):
        return len(self.a_cols) + len(self.b_cols) * (len(self.b_cols[0]) + 3) + 3


def _horner(row, ids, alpha):
    acc = 0
    for i in ids:
        acc = (acc * alpha + row[i]) % P
    return acc


def eval_constraints(cfgs, local, nxt, alpha_pub, delta, sel_first, sel_last, sel_trans) -> List[int]:
    """Concrete-value restatement of LineaAIR::eval: the constraint list in
    eval order, each already multiplied by its selector (FilteredAirBuilder)."""
    out = []
    for c in cfgs:
        if isinstance(c, PermCfg):   # air/src/lib.rs:116-167
            a_l = (_horner(local, c.a_cols, alpha_pub) + delta) % P
            b_l = (_horner(local, c.b_cols, alpha_pub) + delta) % P
            out.append((b_l * local[c.b_inv] - 1) % P)
            out.append(sel_first * (local[c.check] - a_l * local[c.b_inv]) % P)
            a_n = (_horner(nxt, c.a_cols, alpha_pub) + delta) % P
            out.append(sel_trans * (nxt[c.check] - local[c.check] * a_n % P * nxt[c.b_inv]) % P)
            out.append(sel_last * (local[c.check] - 1) % P)
        else:                          # air/src/lib.rs:57-114
            a_l = (_horner(local, c.a_cols, alpha_pub) + delta) % P
            out.append((a_l * local[c.a_inv] - 1) % P)
            lc = local[c.a_filter] * local[c.a_inv] % P
            nc = nxt[c.a_filter] * nxt[c.a_inv] % P
            for t, bids in enumerate(c.b_cols):
                b_l = (_horner(local, bids, alpha_pub) + delta) % P
                out.append((b_l * local[c.b_inv[t]] - 1) % P)
                lc = (lc - local[c.b_filter[t]] * local[c.occ[t]] % P * local[c.b_inv[t]]) % P
                nc = (nc - nxt[c.b_filter[t]] * nxt[c.occ[t]] % P * nxt[c.b_inv[t]]) % P
            out.append(sel_first * (local[c.check] - lc) % P)
            out.append(sel_trans * ((nxt[c.check] - local[c.check]) - nc) % P)
            out.append(sel_last * local[c.check] % P)
    return out


def constraint_degrees(cfgs, public_degree: int = 1) -> List[int]:
    """Symbolic degree_multiple of each constraint (p3-uni-stark symbolic
    rules; U6 ``public_degree``: 1 = the fork rule bench.log implies, 0 =
    upstream).  Main-trace variables 1, constants 0, IsFirstRow/IsLastRow 1,
    IsTransition 0; Add/Sub = max, Mul = sum."""
    pd = public_degree

    def horner_deg(n):
        d = 0  # starts from the constant ZERO
        for _ in range(n):
            d = max(d + pd, 1)
        return d

    out = []
    for c in cfgs:
        if isinstance(c, PermCfg):
            a = max(horner_deg(len(c.a_cols)), pd)
            b = max(horner_deg(len(c.b_cols)), pd)
            out.append(max(b + 1, 0))                 # b_chal * b_inv - 1
            out.append(1 + max(1, a + 1))             # first * (check - a*binv)
            out.append(0 + max(1, 1 + a + 1))         # trans * (check' - check*a'*binv')
            out.append(1 + max(1, 0))                 # last * (check - 1)
        else:
            a = max(horner_deg(len(c.a_cols)), pd)
            out.append(a + 1)
            lc = 2
            for bids in c.b_cols:
                b = max(horner_deg(len(bids)), pd)
                out.append(b + 1)
                lc = max(lc, 3)
            out.append(1 + max(1, lc))
            out.append(0 + max(1, lc))
            out.append(1 + 1)
    return out


def log_quotient_degree(cfgs, public_degree: int = 1) -> int:
    d = max(max(constraint_degrees(cfgs, public_degree)), 2)
    return log2_ceil(d - 1)


# ---------------------------------------------------------------------------
# Witness generation (trace/src/permutation.rs:24-93, trace/src/lookup.rs:46-176,
# trace/src/lib.rs:62-106) -- used to build valid synthetic traces.
# ---------------------------------------------------------------------------
def perm_witness(a: List[List[int]], b: List[List[int]], alpha: int, delta: int):
    """Columns appended in order a.., b.., b_inverse, check."""
    sz = len(a[0])
    binv, chk = [], []
    prev = 1
    for i in range(sz):
        ac = _horner([col[i] for col in a], range(len(a)), alpha)
        bc = _horner([col[i] for col in b], range(len(b)), alpha)
        bi = inv(bc + delta)
        binv.append(bi)
        prev = prev * (ac + delta) % P * bi % P
        chk.append(prev)
    assert chk[-1] == 1, "failed to check constrain: check column should be 1 on the last row"
    w = len(a)
    cfg = PermCfg(list(range(w)), list(range(w, 2 * w)), 2 * w, 2 * w + 1)
    return cfg, [list(c) for c in a] + [list(c) for c in b] + [binv, chk]


def lookup_witness(a, b, a_filter, b_filter, alpha, delta):
    """a: list of cols; b: list of tables, each a list of cols."""
    sz = len(a[0])
    occ = {}
    for i in range(sz):
        if a_filter[i] == 0:
            continue
        ac = _horner([col[i] for col in a], range(len(a)), alpha)
        occ[ac] = occ.get(ac, 0) + 1
    a_inv = []
    b_inv = [[] for _ in b]
    mult = [[] for _ in b]
    psum = []
    s = 0
    for i in range(sz):
        ac = _horner([col[i] for col in a], range(len(a)), alpha)
        ai = inv(ac + delta)
        a_inv.append(ai)
        if a_filter[i] != 0:
            s = (s + ai) % P
        for t, tab in enumerate(b):
            bc = _horner([col[i] for col in tab], range(len(tab)), alpha)
            bi = inv(bc + delta)
            b_inv[t].append(bi)
            o = 0
            if bc in occ and b_filter[t][i] != 0:
                o = occ.pop(bc)
                s = (s - bi * o) % P
            mult[t].append(o)
        psum.append(s)
    assert psum[-1] == 0, "failed to check constrain: check column should be 0 on the last row"
    na, nt, nbc = len(a), len(b), len(b[0])
    b_ids = [[na + t * nbc + j for j in range(nbc)] for t in range(nt)]
    a_filter_id = b_ids[-1][-1] + 1
    b_filter_ids = [a_filter_id + 1 + t for t in range(nt)]
    a_inv_id = b_filter_ids[-1] + 1
    b_inv_ids = [a_inv_id + 1 + t for t in range(nt)]
    occ_ids = [b_inv_ids[-1] + 1 + t for t in range(nt)]
    check_id = occ_ids[-1] + 1
    cfg = LookupCfg(list(range(na)), b_ids, a_filter_id, b_filter_ids, a_inv_id, b_inv_ids, occ_ids, check_id)
    cols = [list(c) for c in a]
    for tab in b:
        cols += [list(c) for c in tab]
    cols.append(list(a_filter))
    cols += [list(f) for f in b_filter]
    cols.append(a_inv)
    cols += b_inv
    cols += mult
    cols.append(psum)
    return cfg, cols


def shift_cfg(cfg, s: int):
    if isinstance(cfg, PermCfg):
        return PermCfg([i + s for i in cfg.a_cols], [i + s for i in cfg.b_cols], cfg.b_inv + s, cfg.check + s)
    return LookupCfg([i + s for i in cfg.a_cols], [[i + s for i in t] for t in cfg.b_cols], cfg.a_filter + s,
                     [i + s for i in cfg.b_filter], cfg.a_inv + s, [i + s for i in cfg.b_inv],
                     [i + s for i in cfg.occ], cfg.check + s)


def columns_to_rows(cols: List[List[int]]) -> List[List[int]]:
    """trace/src/lib.rs:94-106: row-major, columns in push order."""
    return [[c[i] for c in cols] for i in range(len(cols[0]))]


def synthetic_perm_trace(log_n: int, ncols: int, alpha: int, delta: int, seed: int,
                         small: bool = False):
    """A = uniform Fr columns, B = A with rows shuffled by a
    seeded Fisher-Yates, witness columns per trace/src/permutation.rs:55-74."""
    n = 1 << log_n
    rng = SplitMix64(seed ^ 0x5452414345)  # "TRACE"
    if small:
        a = [[rng.next_u64() & 0xFFFFFFFF for _ in range(n)] for _ in range(ncols)]
    else:
        a = [[rng.sample_fr() for _ in range(n)] for _ in range(ncols)]
    perm = list(range(n))
    for i in range(n - 1, 0, -1):
        j = rng.below(i + 1)
        perm[i], perm[j] = perm[j], perm[i]
    b = [[col[perm[i]] for i in range(n)] for col in a]
    cfg, cols = perm_witness(a, b, alpha, delta)
    return [cfg], cols


def synthetic_wide_trace(log_n: int, alpha: int, delta: int, seed: int, nlookup=4, na=3, ntab=2, nperm=8,
                         pcols=6):
    """SURVEY 8(d) C3 wide AIR: nlookup LogUp lookups (A rows drawn from ntab
    random tables), then nperm permutation groups; RawTrace push order
    (trace/src/lib.rs:81-89: lookups first).  Returns (cfgs, columns)."""
    n = 1 << log_n
    rng = SplitMix64(seed ^ 0x57494445)  # "WIDE"
    cols, cfgs = [], []
    for _ in range(nlookup):
        b = [[[rng.sample_fr() for _ in range(n)] for _ in range(na)] for _ in range(ntab)]
        a = [[0] * n for _ in range(na)]
        for i in range(n):
            t = rng.below(ntab)
            j = rng.below(n)
            for c in range(na):
                a[c][i] = b[t][c][j]
        cfg, lc = lookup_witness(a, b, [1] * n, [[1] * n for _ in range(ntab)], alpha, delta)
        cfgs.append(shift_cfg(cfg, len(cols)))
        cols += lc
    for _ in range(nperm):
        a = [[rng.sample_fr() for _ in range(n)] for _ in range(pcols)]
        perm = list(range(n))
        for i in range(n - 1, 0, -1):
            j = rng.below(i + 1)
            perm[i], perm[j] = perm[j], perm[i]
        b = [[col[perm[i]] for i in range(n)] for col in a]
        cfg, pc = perm_witness(a, b, alpha, delta)
        cfgs.append(shift_cfg(cfg, len(cols)))
        cols += pc
    return cfgs, cols


# ---------------------------------------------------------------------------
# A9 -- selectors_on_coset; A10 -- quotient_values; A11 -- split_evals
# ---------------------------------------------------------------------------
def batch_inverse(xs: List[int]) -> List[int]:
    return [inv(x) for x in xs]


def selectors_on_coset(log_h: int, log_q_size: int):
    """Trace domain H_h (shift 1), quotient coset GEN * H_Q (p3-commit)."""
    h = 1 << log_h
    Q = 1 << log_q_size
    rate_bits = log_q_size - log_h
    s_pow_n = pow(GENERATOR, h, P)
    g_rate = two_adic_generator(rate_bits)
    evals = [(s_pow_n * pow(g_rate, k, P) - 1) % P for k in range(1 << rate_bits)]
    gq = two_adic_generator(log_q_size)
    xs = [GENERATOR * pow(gq, i, P) % P for i in range(Q)]
    wh = two_adic_generator(log_h)
    last = inv(wh)
    first_sel = [evals[i % len(evals)] * inv(xs[i] - 1) % P for i in range(Q)]
    last_sel = [evals[i % len(evals)] * inv(xs[i] - last) % P for i in range(Q)]
    trans = [(x - last) % P for x in xs]
    inv_z = [inv(evals[i % len(evals)]) for i in range(Q)]
    return first_sel, last_sel, trans, inv_z


def quotient_values(cfgs, lde_rows, log_h, log_q, alpha, pub):
    N = len(lde_rows)
    Q = 1 << (log_h + log_q)
    logQ = log_h + log_q
    assert N >= Q
    view = [lde_rows[bitrev(k, logQ)] for k in range(Q)]   # get_evaluations_on_domain
    first, last, trans, inv_z = selectors_on_coset(log_h, logQ)
    step = 1 << log_q
    out = []
    for i in range(Q):
        cs = eval_constraints(cfgs, view[i], view[(i + step) % Q], pub[0], pub[1],
                              first[i], last[i], trans[i])
        acc = 0
        for c in cs:
            acc = (acc * alpha + c) % P
        out.append(acc * inv_z[i] % P)
    return out


# ---------------------------------------------------------------------------
# A12-A15 -- TwoAdicFriPcs::open + FRI prover (p3-fri), A18 -- prove (p3-uni-stark)
# ---------------------------------------------------------------------------
@dataclass
class FriParams:
    log_blowup: int = 3          # bin/src/main.rs:59
    log_final_poly_len: int = 0  # bin/src/main.rs:60
    num_queries: int = 33        # bin/src/main.rs:61
    proof_of_work_bits: int = 0  # bin/src/main.rs:62
    # transcript conventions of the fork (include/lsp.h lsp_params), defaults first
    observe_log_degree: bool = True       # U7: challenger.observe(log_degree)
    observe_public_values: bool = True    # U7: observe_slice(public_values) before alpha
    observe_opened_values: bool = False   # U7: opened values observed before alpha_fri
    sample_bits_montgomery: bool = False  # U8: sample_bits from the Montgomery form
    observe_final_poly: bool = True       # U12: final polynomial observed before grinding

    def transcript_bits(self) -> int:
        """the C oracle's lo_fri.transcript mask (LO_T_*)"""
        return ((not self.observe_log_degree) * 1 | (not self.observe_public_values) * 2
                | self.observe_opened_values * 4 | self.sample_bits_montgomery * 8 | (not self.observe_final_poly) * 16)


def interpolate_coset(low_rows_bitrev: List[List[int]], shift: int, z: int) -> List[int]:
    """p3-interpolation interpolate_coset over a BitReversedMatrixView."""
    h = len(low_rows_bitrev)
    logh = log2_strict(h)
    rows = reverse_slice_index_bits(low_rows_bitrev)  # natural order
    g = two_adic_generator(logh)
    coset = [shift * pow(g, i, P) % P for i in range(h)]
    scale = [c * inv(z - c) % P for c in coset]
    w = len(rows[0])
    sums = [sum(rows[i][c] * scale[i] for i in range(h)) % P for c in range(w)]
    zh = (pow(z, h, P) - pow(shift, h, P)) % P
    denom = pow(shift, h, P) * h % P
    f = zh * inv(denom) % P
    return [s * f % P for s in sums]


def inverse_denominators(log_n: int, shift: int, points: Sequence[int]) -> List[List[int]]:
    """compute_inverse_denominators of TwoAdicFriPcs::open [EXT p3-fri]:
    per point z, 1/(z - shift * w_N^bitrev(i)) over the bit-reversed coset (reached from
    p3_uni_stark::prove, bin/src/main.rs:80-86)."""
    N = 1 << log_n
    g = two_adic_generator(log_n)
    xs = reverse_slice_index_bits([shift * pow(g, i, P) % P for i in range(N)])
    return [[inv(z - x) for x in xs] for z in points]


def open_reduce(mat_rows, inv_denoms, ys, alpha: int, alpha_pow_offset: int, ro: List[int]) -> int:
    """The reduce-rows step of TwoAdicFriPcs::open [EXT p3-fri] for one
    matrix opened at len(ys) points: ro[i] += off * (sum_c alpha^c y_c - sum_c alpha^c M[i][c])
    * inv[z][i], then off *= alpha^width.  Updates ro in place; returns the new offset."""
    w = len(mat_rows[0])
    apw = [pow(alpha, c, P) for c in range(w)]
    rr = [sum(a * v for a, v in zip(apw, row)) % P for row in mat_rows]
    off = alpha_pow_offset
    for invz, yz in zip(inv_denoms, ys):
        red_ys = sum(a * y for a, y in zip(apw, yz)) % P
        for i in range(len(ro)):
            ro[i] = (ro[i] + off * (red_ys - rr[i]) % P * invz[i]) % P
        off = off * pow(alpha, w, P) % P
    return off


def fold_vector(v: List[int], beta: int) -> List[int]:
    """TwoAdicFriGenericConfig::fold_matrix over RowMajorMatrix(v, 2)."""
    m = len(v) // 2
    logm = log2_strict(m)
    g_inv = inv(two_adic_generator(logm + 1))
    half = inv(2)
    half_beta = beta * half % P
    powers = [half_beta * pow(g_inv, i, P) % P for i in range(m)]
    powers = reverse_slice_index_bits(powers)
    return [((half + powers[i]) * v[2 * i] + (half - powers[i]) * v[2 * i + 1]) % P for i in range(m)]


def fold_row(index: int, log_height: int, beta: int, e0: int, e1: int) -> int:
    sub_start = pow(two_adic_generator(log_height + 1), bitrev(index, log_height), P)
    xs = [sub_start, sub_start * two_adic_generator(1) % P]
    # reverse_slice_index_bits on 2 elements is the identity
    return (e0 + (beta - xs[0]) * (e1 - e0) % P * inv(xs[1] - xs[0])) % P


@dataclass
class Proof:
    degree_bits: int
    log_q: int
    width: int
    trace_root: int
    quotient_root: int
    trace_local: List[int]
    trace_next: List[int]
    quotient_chunks: List[int]
    fri_roots: List[int]
    final_poly: int
    pow_witness: int
    # per query: (trace_row, trace_path, q_row, q_path, [(sibling, path) per round])
    queries: list


def prove(cfgs, trace_rows: List[List[int]], pub: List[int], pp: Poseidon2Params,
          fri: FriParams = FriParams(), public_degree: int = 1, trace_log: dict = None) -> Proof:
    h = len(trace_rows)
    log_h = log2_strict(h)
    w = len(trace_rows[0])
    lb = fri.log_blowup
    log_q = log_quotient_degree(cfgs, public_degree)
    q = 1 << log_q
    nconstraints = len(constraint_degrees(cfgs, public_degree))
    log = trace_log if trace_log is not None else {}

    # commit to trace data: shift = GEN / 1
    lde = coset_lde_batch(trace_rows, lb, GENERATOR)
    t_tree = merkle_commit([lde], pp)
    log["trace_lde"] = lde
    log["trace_layers"] = t_tree.layers

    ch = HashChallenger(pp, mont_bits=fri.sample_bits_montgomery)
    if fri.observe_log_degree:
        ch.observe(log_h)
    ch.observe(t_tree.root)
    if fri.observe_public_values:
        ch.observe_slice(pub)
    alpha = ch.sample()
    log["alpha"] = alpha

    qv = quotient_values(cfgs, lde, log_h, log_q, alpha, pub)
    log["quotient"] = qv
    # split_evals: chunk j = qv[j::q]; as an h x q row-major matrix this is qv itself
    Q = h * q
    gq = two_adic_generator(log_h + log_q)
    chunk_rows = [qv[k * q:(k + 1) * q] for k in range(h)]
    # chunk j domain shift GEN * gq^j -> lde shift GEN / (GEN*gq^j) = gq^-j
    shifts = [inv(pow(gq, j, P)) for j in range(q)]
    q_lde = coset_lde_batch(chunk_rows, lb, shifts)
    q_tree = merkle_commit([[[r[j]] for r in q_lde] for j in range(q)], pp)
    log["quotient_lde"] = q_lde
    log["quotient_layers"] = q_tree.layers
    ch.observe(q_tree.root)
    zeta = ch.sample()
    zeta_next = zeta * two_adic_generator(log_h) % P
    log["zeta"] = zeta

    # ---- TwoAdicFriPcs::open
    N = h << lb
    logN = log_h + lb
    invd = dict(zip((zeta, zeta_next), inverse_denominators(logN, GENERATOR, [zeta, zeta_next])))

    low = lde[:h]
    ys_zeta = interpolate_coset(low, GENERATOR, zeta)
    ys_next = interpolate_coset(low, GENERATOR, zeta_next)
    qlow = q_lde[:h]
    ys_q = interpolate_coset(qlow, GENERATOR, zeta)   # one value per chunk (width-1 matrices)
    if fri.observe_opened_values:  # U7: (matrix, point) order
        ch.observe_slice(ys_zeta + ys_next + ys_q)
    alpha_fri = ch.sample()
    log["alpha_fri"] = alpha_fri

    ro = [0] * N
    off = 1  # alpha_fri^num_reduced
    off = open_reduce(lde, [invd[zeta], invd[zeta_next]], [ys_zeta, ys_next], alpha_fri, off, ro)
    for j in range(q):
        off = open_reduce([[r[j]] for r in q_lde], [invd[zeta]], [[ys_q[j]]], alpha_fri, off, ro)
    log["fri_input"] = list(ro)

    # ---- FRI commit phase
    folded = ro
    fri_trees = []
    betas = []
    final_len = 1 << (lb + fri.log_final_poly_len)
    while len(folded) > final_len:
        tr = merkle_commit([[[folded[2 * i], folded[2 * i + 1]] for i in range(len(folded) // 2)]], pp)
        ch.observe(tr.root)
        beta = ch.sample()
        betas.append(beta)
        fri_trees.append(tr)
        folded = fold_vector(folded, beta)
    fin = reverse_slice_index_bits(folded)
    coeffs = idft(fin)
    final_poly = coeffs[0]
    assert all(c == 0 for c in coeffs[1 << fri.log_final_poly_len:]), "final poly degree too high"
    if fri.observe_final_poly:
        ch.observe(final_poly)
    log["betas"] = betas
    pow_w = ch.grind(fri.proof_of_work_bits)

    queries = []
    for _ in range(fri.num_queries):
        idx = ch.sample_bits(logN)
        t_rows, t_path = merkle_open(t_tree, idx)
        q_rows, q_path = merkle_open(q_tree, idx)
        steps = []
        for r, tr in enumerate(fri_trees):
            ii = idx >> r
            rows, path = merkle_open(tr, ii >> 1)
            steps.append((rows[0][(ii ^ 1) & 1], path))
        queries.append((t_rows[0], t_path, [x[0] for x in q_rows], q_path, steps))

    return Proof(log_h, log_q, w, t_tree.root, q_tree.root, ys_zeta, ys_next, ys_q,
                 [t.root for t in fri_trees], final_poly, pow_w, queries)


def verify(cfgs, proof: Proof, pub: List[int], pp: Poseidon2Params, fri: FriParams = FriParams(),
           public_degree: int = 1) -> bool:
    log_h = proof.degree_bits
    h = 1 << log_h
    w = proof.width
    log_q = log_quotient_degree(cfgs, public_degree)
    if log_q != proof.log_q:
        return False
    q = 1 << log_q
    lb = fri.log_blowup
    logN = log_h + lb
    ch = HashChallenger(pp, mont_bits=fri.sample_bits_montgomery)
    if fri.observe_log_degree:
        ch.observe(log_h)
    ch.observe(proof.trace_root)
    if fri.observe_public_values:
        ch.observe_slice(pub)
    alpha = ch.sample()
    ch.observe(proof.quotient_root)
    zeta = ch.sample()
    wh = two_adic_generator(log_h)
    zeta_next = zeta * wh % P
    if fri.observe_opened_values:
        ch.observe_slice(list(proof.trace_local) + list(proof.trace_next) + list(proof.quotient_chunks))
    alpha_fri = ch.sample()
    betas = []
    for root in proof.fri_roots:
        ch.observe(root)
        betas.append(ch.sample())
    if len(proof.fri_roots) != logN - lb - fri.log_final_poly_len:
        return False
    if fri.observe_final_poly:
        ch.observe(proof.final_poly)
    if not ch.check_witness(fri.proof_of_work_bits, proof.pow_witness):
        return False
    gN = two_adic_generator(logN)
    for (t_row, t_path, q_row, q_path, steps) in proof.queries:
        idx = ch.sample_bits(logN)
        if not merkle_verify(proof.trace_root, idx, [t_row], t_path, pp):
            return False
        if not merkle_verify(proof.quotient_root, idx, [[v] for v in q_row], q_path, pp):
            return False
        x = GENERATOR * pow(gN, bitrev(idx, logN), P) % P
        ro = 0
        apow = 1
        for z, ys, row in ((zeta, proof.trace_local, t_row), (zeta_next, proof.trace_next, t_row)):
            for pz, px in zip(ys, row):
                ro = (ro + apow * (px - pz) % P * inv(x - z)) % P
                apow = apow * alpha_fri % P
        for j in range(q):
            ro = (ro + apow * (q_row[j] - proof.quotient_chunks[j]) % P * inv(x - zeta)) % P
            apow = apow * alpha_fri % P
        folded = ro
        index = idx
        for r, (sib, path) in enumerate(steps):
            log_folded = logN - 1 - r
            evals = [folded, folded]
            evals[(index ^ 1) & 1] = sib
            if not merkle_verify(proof.fri_roots[r], index >> 1, [evals], path, pp):
                return False
            index >>= 1
            folded = fold_row(index, log_folded, betas[r], evals[0], evals[1])
        if folded != proof.final_poly:
            return False
    # out-of-domain quotient identity
    Qlog = log_h + log_q
    gq = two_adic_generator(Qlog)
    shifts = [GENERATOR * pow(gq, i, P) % P for i in range(q)]

    def zp(shift, x):
        return (pow(x * inv(shift) % P, h, P) - 1) % P
    zps = []
    for i in range(q):
        prod = 1
        for j in range(q):
            if j != i:
                prod = prod * zp(shifts[j], zeta) % P * inv(zp(shifts[j], shifts[i])) % P
        zps.append(prod)
    quotient = sum(zps[i] * proof.quotient_chunks[i] for i in range(q)) % P
    z_h = (pow(zeta, h, P) - 1) % P
    first = z_h * inv(zeta - 1) % P
    last = z_h * inv(zeta - inv(wh)) % P
    trans = (zeta - inv(wh)) % P
    cs = eval_constraints(cfgs, proof.trace_local, proof.trace_next, pub[0], pub[1], first, last, trans)
    acc = 0
    for c in cs:
        acc = (acc * alpha + c) % P
    return acc * inv(z_h) % P == quotient


# ---------------------------------------------------------------------------
# Proof serialization (the build's own documented format)
# ---------------------------------------------------------------------------
def serialize_proof(p: Proof) -> bytes:
    fe = to_canon_bytes
    out = bytearray(b"LSPPRF02")
    out += struct.pack("<6I", p.degree_bits, p.log_q, p.width, len(p.queries), len(p.fri_roots), 1)
    out += fe(p.trace_root) + fe(p.quotient_root)
    for v in p.trace_local + p.trace_next + p.quotient_chunks + p.fri_roots:
        out += fe(v)
    out += fe(p.final_poly) + fe(p.pow_witness)
    for (t_row, t_path, q_row, q_path, steps) in p.queries:
        for v in t_row:
            out += fe(v)
        out += struct.pack("<I", len(t_path))
        for v in t_path:
            out += fe(v)
        for v in q_row:
            out += fe(v)
        out += struct.pack("<I", len(q_path))
        for v in q_path:
            out += fe(v)
        for sib, path in steps:
            out += fe(sib)
            out += struct.pack("<I", len(path))
            for v in path:
                out += fe(v)
    return bytes(out)


def deserialize_proof(b: bytes) -> Proof:
    assert b[:8] == b"LSPPRF02"
    off = 8
    degree_bits, log_q, w, nq, nr, nf = struct.unpack_from("<6I", b, off)
    assert nf == 1, "this oracle handles a 1-coefficient final polynomial"
    off += 24

    def fe():
        nonlocal off
        v = int.from_bytes(b[off:off + 32], "little")
        off += 32
        return v

    def u32():
        nonlocal off
        v = struct.unpack_from("<I", b, off)[0]
        off += 4
        return v
    q = 1 << log_q
    t_root, q_root = fe(), fe()
    tl = [fe() for _ in range(w)]
    tn = [fe() for _ in range(w)]
    qc = [fe() for _ in range(q)]
    roots = [fe() for _ in range(nr)]
    fp, pw = fe(), fe()
    queries = []
    for _ in range(nq):
        t_row = [fe() for _ in range(w)]
        t_path = [fe() for _ in range(u32())]
        q_row = [fe() for _ in range(q)]
        q_path = [fe() for _ in range(u32())]
        steps = []
        for _ in range(nr):
            sib = fe()
            steps.append((sib, [fe() for _ in range(u32())]))
        queries.append((t_row, t_path, q_row, q_path, steps))
    assert off == len(b)
    return Proof(degree_bits, log_q, w, t_root, q_root, tl, tn, qc, roots, fp, pw, queries)
