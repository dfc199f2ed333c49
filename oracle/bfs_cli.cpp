// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.hpp).
// CPU baseline driver: `bfs_cli <model> <N> [threads] [target]` runs the restated `spawn_bfs` and
// prints the reference's `report` tail (src/checker.rs:229-238) plus a machine-readable line.
#include <cstdlib>
#include <iostream>

#include "models.hpp"
#include "paxos.hpp"
#include "actor.hpp"

using namespace oracle;

template <class M>
int run(M m, size_t threads, u64 target) {
    CheckerOptions o;
    o.thread_count = threads;
    o.target_state_count = target;
    auto t0 = std::chrono::steady_clock::now();
    BfsChecker<M> c(std::move(m), o);
    c.join();
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << c.report_done();
    std::cout << "RESULT state_count=" << c.state_count() << " unique=" << c.unique_state_count()
              << " max_depth=" << c.max_depth() << " threads=" << threads << " sec=" << sec
              << " unique_per_sec=" << (double)c.unique_state_count() / sec << std::endl;
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::cerr << "usage: bfs_cli <2pc|increment|increment_lock|linear_equation|paxos|single_copy> <N> [threads] [target]\n";
        return 2;
    }
    std::string model = argv[1];
    size_t n = (size_t)std::atoll(argv[2]);
    size_t threads = argc > 3 ? (size_t)std::atoll(argv[3]) : 1;
    u64 target = argc > 4 ? (u64)std::atoll(argv[4]) : 0;
    if (model == "2pc") return run(TwoPhaseSys{n}, threads, target);
    if (model == "increment") return run(Increment{n}, threads, target);
    if (model == "increment_lock") return run(IncrementLock{n}, threads, target);
    if (model == "paxos") return run(paxos::PaxosModel{n, 3}, threads, target);
    if (model == "linear_equation") return run(LinearEquation{2, 4, 7}, threads, target);
    if (model == "single_copy") {  // examples/single-copy-register.rs `check N`: N clients, 1 server
        actor::SingleCopyModel m;
        m.sys.client_count = n;
        m.sys.server_count = 1;
        return run(std::move(m), threads, target);
    }
    std::cerr << "unknown model " << model << "\n";
    return 2;
}
