// A GpuModel outside the engine's registry, built into its own plugin library: the 3x3 sliding
// puzzle of the reference crate's documentation (src/lib.rs:40-116, `struct Puzzle([u8; 9])`).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include \
//         examples/plugins/sliding_puzzle.hip -o examples/plugins/libsliding_puzzle.so -L/opt/rocm/lib -lrccl
//
// State: the 9 cells, 4 bits each (cell i at bits 4i..4i+3), one 64-bit word. Actions, in the
// order `actions()` lists them (lib.rs:55-59): Down, Up, Right, Left; every state lists all four
// and `next_state` is None when the empty cell is on the edge the tile would come from (lib.rs:61-78),
// so `apply` returns false there. Property: sometimes "solved" = [0, 1, ..., 8] (lib.rs:80-87).
#include "stateright_gpu_model.hpp"

using sr::i64;
using sr::u64;

struct SlidingPuzzle {
    static constexpr int W = 1, MW = 1, NPROPS = 1;
    u64 init = 0;

    static constexpr u64 SOLVED = 0x876543210ull;  // cell i holds i

    int max_actions() const { return 4; }
    int max_out_degree() const { return 4; }
    SR_HD static int cell(u64 s, int i) { return (int)(s >> (4 * i) & 15); }
    SR_HD static int empty(u64 s) {
        int e = 0;
        for (int i = 0; i < 9; ++i)
            if (cell(s, i) == 0) e = i;
        return e;
    }
    SR_HD void enabled(const u64*, u64* m) const { m[0] = 15; }
    SR_HD bool apply(const u64* sp, int a, u64* o) const {
        const u64 s = sp[0];
        const int e = empty(s), y = e / 3, x = e % 3;
        int from;
        switch (a) {
            case 0: if (y == 0) return false; from = e - 3; break;  // Down: the tile above moves down
            case 1: if (y == 2) return false; from = e + 3; break;  // Up: the tile below moves up
            case 2: if (x == 0) return false; from = e - 1; break;  // Right: the tile on the left
            default: if (x == 2) return false; from = e + 1; break; // Left: the tile on the right
        }
        const u64 tile = (u64)cell(s, from);
        o[0] = (s & ~(15ull << (4 * e)) & ~(15ull << (4 * from))) | tile << (4 * e);
        return true;
    }
    SR_HD bool discovers(int, const u64* s) const { return s[0] == SOLVED; }

    int init_states(u64* out) const {
        out[0] = init;
        return 1;
    }
    int expectation(int) const { return sr::SOMETIMES; }
    const char* prop_name(int) const { return "solved"; }
    int describe_width() const { return 9; }
    void describe(const u64* s, i64* d) const {
        for (int i = 0; i < 9; ++i) d[i] = cell(s[0], i);
    }
    void undescribe(const i64* d, u64* s) const {
        s[0] = 0;
        for (int i = 0; i < 9; ++i) s[0] |= ((u64)d[i] & 15) << (4 * i);
    }
    i64 action_id(const u64*, int a) const { return a; }
    std::string action_name(i64 id) const {
        static const char* names[] = {"Down", "Up", "Right", "Left"};
        return id >= 0 && id < 4 ? names[id] : "?";
    }
    i64 action_id_bound() const { return 4; }
};

static SlidingPuzzle make_puzzle(const int64_t* p, int32_t n, int /*device*/) {
    if (n != 9) throw sr::Error(SR_ERR_ARG, "sliding_puzzle: 9 cells expected");
    SlidingPuzzle m;
    int seen = 0;
    for (int i = 0; i < 9; ++i) {
        if (p[i] < 0 || p[i] > 8 || (seen >> p[i] & 1)) throw sr::Error(SR_ERR_ARG, "sliding_puzzle: cells must be a permutation of 0..8");
        seen |= 1 << p[i];
        m.init |= (u64)p[i] << (4 * i);
    }
    return m;
}

SR_GPU_PLUGIN(sliding_puzzle, SlidingPuzzle, make_puzzle)
