"""The exchange calibration measures what the sharded proofs do.

lsp_comm_selftest times this GPU's inverse NTT (lsp_calibrate_intt) and the
sharded proofs choose their exchange on that rate.  Round 5 timed the inverse
on an all-zero buffer; this chip is power-held on MAD-dense work and zero
operands draw less power, so that probe could overstate the rate.  The probe
now runs on seeded random field elements, and here it must agree within 10 %
with the trace-inverse phase of a real sharded proof at the same shape (and
within 20 % at the wider shape the self-test probes): rank 0
of a 2-rank proof of the 3x3 AIR at 2^20 rows (loopback transport, so the
rank runs alone on the GPU) inverts its w/G = 4 columns of 2^20 as one phase
("trace inverse NTT", device events).
"""
import statistics

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_intt_probe_matches_the_proofs_inverse_phase(gpu_ctx, monkeypatch):
    import ctypes
    from linea_stark_prover_amd import _lib as L
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, _take_proof

    log_n, G = 20, 2
    h, w = 1 << log_n, 8
    cg = w // G
    monkeypatch.setenv("LSP_SHARD_SPLIT_INTT", "1")  # the split: the inverse is a phase of its own
    with Context(gpu_ctx.config) as ctx:
        rate_shape = ctx.calibrate_intt(log_n, cg)   # the phase's own shape (G elem/s)
        rate_attach = ctx.calibrate_intt(20, 8)      # the shape lsp_comm_selftest probes
        L.check(L.lib().lsp_ctx_attach_loopback(ctx.h, 0, G), ctx.h)
        a, d, _ = ctx.config.seeded()
        pub = np.ascontiguousarray(np.concatenate([a, d]))
        dt = ctx.gen_permutation_trace_device(log_n, 3, a, d)
        ctx.set_phase_timing(True, only=["trace inverse NTT"])
        desc = permutation_air(3).descriptor()
        desc = (ctypes.c_int32 * len(desc))(*desc)
        ms = []
        for i in range(6):  # one warm-up
            pf = ctypes.c_void_p()
            ctx._chk(L.lib().lsp_prove_sharded(ctx.h, dt, h, w, desc, len(desc), pub.ctypes.data, 2,
                                               L.LSP_MEM_DEVICE, ctypes.byref(pf)))
            _take_proof(pf, size_only=True)
            if i:
                ms += [v for k, v in ctx.last_timings() if k == "trace inverse NTT"]
        ctx.dev_free(dt)
    assert len(ms) == 5, ms
    phase_rate = h * cg / (statistics.median(ms) * 1e-3) / 1e9
    print(f"inverse NTT: probe {rate_shape:.3f} (2^20 x 4), {rate_attach:.3f} (2^20 x 8), "
          f"proof phase {phase_rate:.3f} G elem/s")
    assert abs(rate_shape / phase_rate - 1) < 0.10, (rate_shape, phase_rate)
    # the probe lsp_comm_selftest runs is 8 columns wide, the phase 4: a wider
    # matrix inverts faster per element (+3 .. +12 % on the boxes seen), so the
    # attach-shape figure gets a looser bound than the same-shape one
    assert abs(rate_attach / phase_rate - 1) < 0.20, (rate_attach, phase_rate)


def test_box_speed_stamp(gpu_ctx):
    """bench.py's box-speed stamp on the GPU: the SMU's engine clock sampled
    while proofs run (amdsmi gpu_metrics, the device matched by bus id), the
    full-occupancy permutation probe and the host compression rate"""
    import os
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    s = bench.ClockSampler(gpu_ctx.device, period=0.01)
    assert s.status == "ok", s.status
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(14, 3, a, d)
    pub = np.concatenate([a, d])
    s.start()
    t = time.time()
    while time.time() - t < 0.3:
        gpu_ctx.prove(tr, permutation_air(3), pub)
    got = s.stop()
    assert got is not None and got["samples"] >= 5, got
    assert 500 < got["sclk_mhz_mean"] < 3000 and got["sclk_mhz_min"] <= got["sclk_mhz_max"], got
    box = bench.box_speed(gpu_ctx, got, s.status, 60.0)
    assert box["gpu_perm_mperm_per_s"] > 100 and box["host_compress_k_per_s"] > 10
    assert abs(box["ms_per_step_x_sclk_ghz"] - 60.0 * got["sclk_mhz_mean"] / 1e3) < 1e-9
