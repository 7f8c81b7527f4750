// uttt_bits.h — Ultimate Tic-Tac-Toe rules on packed bitboards, compiled for
// both the host (State API) and gfx950 (search kernels).
//
// Semantics follow cpp/uttt_game.cpp exactly, including its quirks:
//   * a full small board with no winner closes for BOTH sides (uttt_game.cpp:117-128),
//   * is_lose inspects only the opponent's main board (uttt_game.cpp:77-79),
//   * next() places the stone unvalidated (uttt_game.cpp:97-145).
// Layout: uttt_state_t (include/uttt_engine.h). Action a = board*9 + cell sits
// at bit a % 27 of word a / 27, so ascending bit order == ascending action order
// == the reference's legal_actions() order (uttt_game.cpp:158-188).
#pragma once

#include <stdint.h>

#include "uttt_engine.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define UTTT_HD __host__ __device__ __forceinline__
#else
#define UTTT_HD static inline
#endif

namespace uttt {

constexpr uint32_t kCells = 0x1FFu;         // 9 cells of one small board
constexpr uint32_t kWord = 0x7FFFFFFu;      // 27 cells (3 boards) per word
constexpr uint64_t kGold = 0x9E3779B97F4A7C15ull;

UTTT_HD uint32_t popc32(uint32_t x) { return (uint32_t)__builtin_popcount(x); }

// Division of small non-negative ints by 9, 27 and 3 as one 24-bit multiply and a shift: exact for
// 0..511 (tests/test_host_api.py checks every value); the general forms are 32-bit mul_hi sequences,
// a quarter-rate instruction each, on the descent's critical path.
UTTT_HD int div9(int a) { return (a * 57) >> 9; }
UTTT_HD int div27(int a) { return (a * 19) >> 9; }
UTTT_HD int div3(int a) { return (a * 171) >> 9; }

// 3-in-a-row on a 9-bit board (uttt_game.cpp:35-61: rows, columns, diagonals): a row is full when
// bits i, i+1, i+2 are (i = 0, 3, 6), a column when i, i+3, i+6 are (i = 0, 1, 2); the diagonals 0x111,
// 0x054 by compares. Equal to the eight compares of the reference for all 512 masks (tests).
UTTT_HD bool win9(uint32_t m) {
    return ((m & (m >> 1) & (m >> 2) & 0x049u) | (m & (m >> 3) & (m >> 6) & 0x007u)) != 0u ||
           (m & 0x111u) == 0x111u || (m & 0x054u) == 0x054u;
}

UTTT_HD uint32_t main_own(const uttt_state_t &s) { return s.mains & kCells; }
UTTT_HD uint32_t main_opp(const uttt_state_t &s) { return (s.mains >> 16) & kCells; }
UTTT_HD uint32_t cells_of(uint32_t word, int b) { return (word >> (9 * (b - 3 * div3(b)))) & kCells; }

UTTT_HD bool is_lose(const uttt_state_t &s) { return win9(main_opp(s)); }

// Boards a move may go to (uttt_game.cpp:158-181).
UTTT_HD uint32_t candidate_boards(const uttt_state_t &s) {
    const uint32_t open = ~(main_own(s) | main_opp(s)) & kCells;
    if (s.active >= 0 && ((open >> s.active) & 1u)) return 1u << s.active;
    return open;
}

// Legal-move mask in action order (uttt_game.cpp:148-191).
UTTT_HD void legal_mask(const uttt_state_t &s, uint32_t m[3]) {
    m[0] = m[1] = m[2] = 0u;
    if (is_lose(s)) return;
    const uint32_t cand = candidate_boards(s);
#pragma unroll
    for (int w = 0; w < 3; ++w) {
        uint32_t boards = 0u;
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if ((cand >> (3 * w + j)) & 1u) boards |= kCells << (9 * j);
        m[w] = ~(s.own[w] | s.opp[w]) & boards & kWord;
    }
}

UTTT_HD uint32_t legal_count(const uttt_state_t &s) {
    uint32_t m[3];
    legal_mask(s, m);
    return popc32(m[0]) + popc32(m[1]) + popc32(m[2]);
}

// is_done = is_lose || no legal move (uttt_game.cpp:82-89).
UTTT_HD bool is_done(const uttt_state_t &s) { return is_lose(s) || legal_count(s) == 0u; }

UTTT_HD bool is_first_player(const uttt_state_t &s) {  // uttt_game.cpp:92-94
    return popc32(s.own[0]) + popc32(s.own[1]) + popc32(s.own[2]) ==
           popc32(s.opp[0]) + popc32(s.opp[1]) + popc32(s.opp[2]);
}

// State::next (uttt_game.cpp:97-145): sides swap, the mover's stone lands in
// the new opponent set; a won small board sets the new opponent's main bit, a
// full one sets both; the next active board is the cell unless it is closed.
UTTT_HD uttt_state_t next_state(const uttt_state_t &s, int a) {
    const int b = div9(a), c = a - 9 * b, w = div27(a);
    uttt_state_t n;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        n.own[i] = s.opp[i];
        n.opp[i] = s.own[i];
    }
    uint32_t mown = main_opp(s), mopp = main_own(s);
    // word w chosen by selects, not a dynamic index into the local arrays (which the device
    // compiler may place in scratch)
    const uint32_t bit = 1u << (a - 27 * w);
    n.opp[0] |= w == 0 ? bit : 0u;
    n.opp[1] |= w == 1 ? bit : 0u;
    n.opp[2] |= w == 2 ? bit : 0u;
    const uint32_t opp_w = w == 0 ? n.opp[0] : (w == 1 ? n.opp[1] : n.opp[2]);
    const uint32_t own_w = w == 0 ? n.own[0] : (w == 1 ? n.own[1] : n.own[2]);
    const uint32_t eb = cells_of(opp_w, b);
    if (win9(eb)) {
        mopp |= 1u << b;
    } else if ((cells_of(own_w, b) | eb) == kCells) {
        mown |= 1u << b;
        mopp |= 1u << b;
    }
    n.mains = mown | (mopp << 16);
    n.active = (((mown | mopp) >> c) & 1u) ? -1 : c;
    return n;
}

// Position of action a's cell in the 9x9 image (uttt_game.cpp:256-257).
UTTT_HD int image_index(int a) {
    const int b = a / 9, c = a % 9;
    return ((b / 3) * 3 + c / 3) * 9 + (b % 3) * 3 + c % 3;
}
// Inverse: image position (R*9+C) -> action.
UTTT_HD int action_at(int pos) {
    const int R = pos / 9, C = pos % 9;
    return ((R / 3) * 3 + C / 3) * 9 + (R % 3) * 3 + C % 3;
}
// the word chosen by selects, not a dynamic index (which puts a local state in LDS or scratch)
UTTT_HD uint32_t bit_of(const uint32_t w[3], int a) {
    const int i = div27(a);
    const uint32_t x = i == 0 ? w[0] : (i == 1 ? w[1] : w[2]);
    return (x >> (a - 27 * i)) & 1u;
}

// ---------------------------------------------------------------------------
// Deterministic hash evaluator (DESIGN.md "Hash evaluator"). Input: the 243
// bits of the NCHW network input, bit j = ch*81 + R*9 + C, packed into 4 u64.
// ---------------------------------------------------------------------------
UTTT_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

UTTT_HD uint64_t hash_words(const uint64_t x[4]) {
    uint64_t h = kGold;
#pragma unroll
    for (int i = 0; i < 4; ++i) h = mix64(h ^ x[i]);
    return h;
}

UTTT_HD float hash_prior(uint64_t h, int a) {
    const uint32_t mode = (uint32_t)((h >> 8) & 15u);
    const uint64_t r = mix64(h + (uint64_t)(a + 1) * kGold);
    float p = (float)(uint32_t)(r >> 40) * (1.0f / 16777216.0f);
    if (mode == 0u) p = 0.0f;
    else if (mode == 1u) p = p * 0x1p-140f;  // subnormal priors: catches flush-to-zero
    else if (mode == 2u && (a & 3)) p = 0.0f;
    return p;
}

UTTT_HD float hash_value(uint64_t h) {
    const uint64_t r = mix64(h ^ 0xD6E8FEB86659FD93ull);
    return (float)((int32_t)(r % 2001ull) - 1000) / 1000.0f;
}

}  // namespace uttt
