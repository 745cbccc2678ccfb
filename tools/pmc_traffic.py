"""Per-coset_lde_batch HBM traffic from the rocprofv3 --pmc passes of
tools/pmc_round.sh (FETCH_SIZE and WRITE_SIZE in separate passes, KB units).
gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes
of wide coalesced streaming reads -> doubled; WRITE_SIZE taken as is.
Writes a JSON summary for the last (steady-state) LDE call."""
import csv, json, os, sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from linea_stark_prover_amd.build import library_hash, source_hash

def run_stamp(run_dir):
    """the library stamp the box recorded for this run (tools/pmc_stamp.sh
    copies liblsp_hip.so.src there), else the local library's"""
    f = os.path.join(run_dir, "lib_src_sha16.txt")
    if os.path.exists(f):
        return open(f).read().strip()
    return library_hash() or source_hash()


def per_dispatch(path):
    out = {}
    for r in csv.DictReader(open(path)):
        k = int(r['Dispatch_Id'])
        out.setdefault(k, [r['Kernel_Name'], 0.0])
        out[k][1] += float(r['Counter_Value'])
    return out

def calls(d):
    """group dispatches into LDE calls: a call is its twist-table kernel (k_pow_tables)
    followed by the NTT passes (k_ntt_rm), up to the next call"""
    ks = sorted(d)
    # a call starts at its first inverse pass (k_ntt_rm<false, 1, ...>: PASS_INV_FIRST),
    # or at the twist-table kernels right before it (absent once the tables are cached)
    starts = []
    for i, k in enumerate(ks):
        if 'k_ntt_rm<false, 1' in d[k][0]:
            j = i
            while j > 0 and any(x in d[ks[j - 1]][0] for x in ('k_pow_tables', 'k_to_f29form')):
                j -= 1
            starts.append(ks[j])
    out = []
    for i, s in enumerate(starts):
        end = starts[i + 1] if i + 1 < len(starts) else ks[-1] + 1
        body = [k for k in ks if s <= k < end and 'copyBuffer' not in d[k][0]]
        if any('k_ntt_rm' in d[k][0] for k in body):
            out.append((body[0], body[-1]))
    return out

fetch = per_dispatch(sys.argv[1]); write = per_dispatch(sys.argv[2])
h, w, added = int(sys.argv[3]), int(sys.argv[4]), 3
lo, hi = calls(fetch)[-1]
kern = [k for k in sorted(fetch) if lo <= k <= hi and 'copyBuffer' not in fetch[k][0]]
fb = sum(fetch[k][1] for k in kern) * 1024 * 2
wb = sum(write[k][1] for k in kern if k in write) * 1024
alg = 32 * w * (h + (h << added))
res = {"kernel": "coset_lde_batch (row-major: inverse DIT pass(es), the fused inverse-last / twisted forward-first pass, in-place forward DIF pass(es))",
       "h": h, "w": w, "fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb,
       "algorithmic_bytes": alg, "traffic_over_algorithmic": (fb + wb) / alg,
       "per_kernel": [{"dispatch": k, "kernel": fetch[k][0].replace('lsp::(anonymous namespace)::', '').replace('void ', '').split('(')[0],
                       "fetch_bytes_x2": fetch[k][1] * 2048, "write_bytes": write.get(k, [0, 0])[1] * 1024}
                      for k in kern],
       "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE separate passes on tools/lde_probe.py; FETCH x2 (gfx950)",
       "lib_src_sha16": run_stamp(os.path.dirname(os.path.dirname(os.path.abspath(sys.argv[1]))))}
print(json.dumps(res, indent=1))
