// Host Poseidon2 permutation: generic 8x32-bit path (poseidon2.hpp) vs the
// 64-bit lazily reduced one the prover uses (poseidon2_host64.hpp); checks
// they agree and times both.
// Build: hipcc --cuda-host-only -O3 -std=c++17 -Ilinea_stark_prover_amd/csrc \
//        tools/ubench/host_perm.cpp -o /tmp/host_perm
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "poseidon2_host64.hpp"
using namespace lsp;

static Fr rnd(std::mt19937_64& g) {
    Fr x;
    for (int j = 0; j < 8; ++j) x.v[j] = (uint32_t)g();
    x.v[7] &= 0x0fffffffu;  // < r
    return x;
}

int main() {
    std::mt19937_64 g(7);
    std::vector<Fr> rc(46);
    for (auto& c : rc) c = rnd(g);
    P2Layout L{8, 22, 11};
    int bad = 0;
    for (int it = 0; it < 1000; ++it) {
        Fr a = rnd(g), b = rnd(g), c = rnd(g), x = a, y = b, z = c;
        permute3_rt(a, b, c, rc.data(), L);
        hp64::permute3_rt(x, y, z, rc.data(), L);
        for (int j = 0; j < 8; ++j) bad += (a.v[j] != x.v[j]) + (b.v[j] != y.v[j]) + (c.v[j] != z.v[j]);
    }
    Fr s0 = rc[1], s1 = rc[2], s2 = rc[3];
    const int N = 20000;
    double us[2];
    for (int v = 0; v < 2; ++v) {
        auto t = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) v ? hp64::permute3_rt(s0, s1, s2, rc.data(), L) : permute3_rt(s0, s1, s2, rc.data(), L);
        us[v] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count() / N;
    }
    printf("host permutation: generic %.2f us, 64-bit lazy %.2f us, mismatches %d (%08x)\n", us[0], us[1], bad, s0.v[0]);
    return bad != 0;
}
