// Host Poseidon2 permutation: generic 8x32-bit path (poseidon2.hpp) vs the
// 64-bit lazily reduced one the prover uses (poseidon2_host64.hpp); checks
// they agree and times both.
// Build: hipcc --cuda-host-only -O3 -std=c++17 -Ilinea_stark_prover_amd/csrc \
//        tools/ubench/host_perm.cpp -o /tmp/host_perm
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "host.hpp"
using namespace lsp;

static Fr rnd(std::mt19937_64& g) {
    Fr x;
    for (int j = 0; j < 8; ++j) x.v[j] = (uint32_t)g();
    x.v[7] &= 0x0fffffffu;  // < r
    return x;
}

int bench_ifma();
int main() {
#ifdef LSP_BENCH_IFMA
    if (bench_ifma()) return 1;
#endif
    std::mt19937_64 g(7);
    std::vector<Fr> rc(46);
    for (auto& c : rc) c = rnd(g);
    P2Layout L{8, 22, 11};
    int bad = 0;
    for (int it = 0; it < 1000; ++it) {
        Fr a = rnd(g), b = rnd(g), c = rnd(g), x = a, y = b, z = c;
        permute3<11>(a, b, c, rc.data(), 8, 22);
        hp64::permute3_rt(x, y, z, rc.data(), L);
        for (int j = 0; j < 8; ++j) bad += (a.v[j] != x.v[j]) + (b.v[j] != y.v[j]) + (c.v[j] != z.v[j]);
    }
    Fr s0 = rc[1], s1 = rc[2], s2 = rc[3];
    const int N = 20000;
    double us[2];
    for (int v = 0; v < 2; ++v) {
        auto t = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) v ? hp64::permute3_rt(s0, s1, s2, rc.data(), L) : permute3<11>(s0, s1, s2, rc.data(), 8, 22);
        us[v] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count() / N;
    }
    printf("host permutation: generic %.2f us, 64-bit lazy %.2f us, mismatches %d (%08x)\n", us[0], us[1], bad, s0.v[0]);
    return bad != 0;
}

// IFMA batch (tools/ubench: build with host_ifma.cpp, see the header comment):
// latency of one 8-lane compression vs one scalar compression
#ifdef LSP_BENCH_IFMA
#include <vector>
int bench_ifma() {
    std::mt19937_64 g(9);
    std::vector<Fr> rc(46);
    for (auto& c : rc) c = rnd(g);
    P2Layout L{8, 22, 11};
    if (!ifma::available()) { printf("no avx512ifma\n"); return 0; }
    std::vector<ifma::Lane8> rc8;
    ifma::prepare(rc, rc8);
    P2Host p{L, rc, {}};
    P2Host q{L, rc, rc8};
    Fr in[16], out[8], ref[8];
    for (auto& x : in) x = rnd(g);
    p.compress_range(in, ref, 0, 8);
    q.compress_range(in, out, 0, 8);
    int bad = 0;
    for (int j = 0; j < 8; ++j) bad += !fr_eq(out[j], ref[j]);
    const int N = 20000;
    auto t = std::chrono::steady_clock::now();
    for (int i = 0; i < N; ++i) { q.compress_range(in, out, 0, 8); in[0] = out[3]; }
    double us8 = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count() / N;
    t = std::chrono::steady_clock::now();
    for (int i = 0; i < N; ++i) { in[0] = p.compress(in[0], in[1]); }
    double us1 = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count() / N;
    printf("host compression: scalar %.2f us each; IFMA %.2f us per 8 (%.2f us each), mismatches %d\n", us1, us8, us8 / 8, bad);
    // 16 lanes (two states in lockstep), every count 1..16
    Fr in2[32], o16[16], r16[16];
    for (auto& x : in2) x = rnd(g);
    for (int n = 1; n <= 16; ++n) {
        for (auto& x : o16) x = fr_zero();
        p.compress_range(in2, r16, 0, n);
        ifma::compress16(in2, in2 + 1, 2, o16, n, rc8, L);
        for (int j = 0; j < n; ++j) bad += !fr_eq(o16[j], r16[j]);
    }
    t = std::chrono::steady_clock::now();
    for (int i = 0; i < N; ++i) { ifma::compress16(in2, in2 + 1, 2, o16, 16, rc8, L); in2[0] = o16[3]; }
    double us16 = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count() / N;
    printf("IFMA x16: %.2f us per 16 (%.2f us each), mismatches %d\n", us16, us16 / 16, bad);
    return bad;
}
#endif
