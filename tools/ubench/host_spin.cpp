// Latency of the host's sequential permutations (transcript samples, tree-top
// chains) while the host pool's workers spin-wait for their next job (`pause`
// loops, HostPool::loop) against workers that sleep.  On a CPU share of SMT
// siblings a spinning sibling takes issue slots from the main thread.
// Prints the process's CPUs and their SMT siblings, then the chain's time per
// permutation with 0 / N spinning / N sleeping helper threads.
// Build: tools/ubench/build.sh host_spin
#include <sched.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <fstream>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "host.hpp"
using namespace lsp;

static Fr rnd(std::mt19937_64& g) {
    Fr x;
    for (int j = 0; j < 8; ++j) x.v[j] = (uint32_t)g();
    x.v[7] &= 0x0fffffffu;
    return x;
}

static double chain_us(const std::vector<Fr>& rc, const P2Layout& L, int n) {
    Fr s0 = rc[1], s1 = rc[2], s2 = rc[3];
    const auto t = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) hp64::permute3_rt(s0, s1, s2, rc.data(), L);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count() / n;
    if (s0.v[0] == 0x12345678u) std::printf("!");
    return us;
}

int main(int argc, char** argv) {
    cpu_set_t cs;
    CPU_ZERO(&cs);
    sched_getaffinity(0, sizeof cs, &cs);
    const int ncpu = CPU_COUNT(&cs);
    std::printf("CPUs in this process's affinity: %d\n", ncpu);
    int shown = 0;
    for (int c = 0; c < CPU_SETSIZE && shown < 4; ++c) {
        if (!CPU_ISSET(c, &cs)) continue;
        std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/thread_siblings_list");
        std::string s;
        std::getline(f, s);
        std::printf("  cpu %d siblings %s\n", c, s.c_str());
        ++shown;
    }
    const int helpers = argc > 1 ? std::atoi(argv[1]) : std::min(15, ncpu - 1);
    std::mt19937_64 g(7);
    std::vector<Fr> rc(46);
    for (auto& c : rc) c = rnd(g);
    const P2Layout L{8, 22, 11};
    const int N = 3000;
    chain_us(rc, L, 500);  // warm
    std::vector<double> alone, spin, sleep;
    for (int rep = 0; rep < 5; ++rep) {
        alone.push_back(chain_us(rc, L, N));
        {
            std::atomic<bool> stop{false};
            std::vector<std::thread> th;
            for (int i = 0; i < helpers; ++i)
                th.emplace_back([&] {
                    while (!stop.load(std::memory_order_relaxed)) __builtin_ia32_pause();
                });
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            spin.push_back(chain_us(rc, L, N));
            stop = true;
            for (auto& t : th) t.join();
        }
        {
            std::mutex m;
            std::condition_variable cv;
            bool stop = false;
            std::vector<std::thread> th;
            for (int i = 0; i < helpers; ++i)
                th.emplace_back([&] {
                    std::unique_lock<std::mutex> lk(m);
                    cv.wait(lk, [&] { return stop; });
                });
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            sleep.push_back(chain_us(rc, L, N));
            {
                std::lock_guard<std::mutex> lk(m);
                stop = true;
            }
            cv.notify_all();
            for (auto& t : th) t.join();
        }
    }
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    std::printf("sequential permutation, %d helper threads: alone %.2f us, helpers spinning %.2f us, helpers asleep %.2f us"
                " (medians of 5 x %d)\n",
                helpers, med(alone), med(spin), med(sleep), N);
    return 0;
}
