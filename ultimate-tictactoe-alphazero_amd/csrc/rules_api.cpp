// rules_api.cpp — host side of the C ABI: one position at a time, the value
// type behind `uttt_cpp.State` (cpp/python_bindings.cpp:53-74). Same bitboard
// code the kernels use (uttt_bits.h).
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "uttt_bits.h"
#include "uttt_engine.h"

namespace uttt {
// Last error of the calling thread, for every entry point of the C ABI (uttt_last_error).
// Kept in this host-only file so the rules build on their own (tests/asan).
static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}
}  // namespace uttt

using namespace uttt;

extern "C" {

const char *uttt_last_error(void) { return g_err.c_str(); }

void uttt_state_initial(uttt_state_t *out) {
    std::memset(out, 0, sizeof(*out));
    out->active = -1;
}

int uttt_state_from_arrays(const int32_t pieces[81], const int32_t enemy[81], const int32_t main_p[9],
                           const int32_t main_e[9], int32_t active, uttt_state_t *out) {
    if (!pieces || !enemy || !main_p || !main_e || !out) {
        set_error("uttt_state_from_arrays: null pointer");
        return UTTT_ERR_ARG;
    }
    if (active < -1 || active > 8) {
        set_error("active_board must be -1..8 (got %d)", active);
        return UTTT_ERR_ARG;
    }
    uttt_state_t s;
    std::memset(&s, 0, sizeof(s));
    for (int a = 0; a < 81; ++a) {
        if ((uint32_t)pieces[a] > 1u || (uint32_t)enemy[a] > 1u) {
            set_error("pieces/enemy_pieces cells must be 0 or 1 (board %d cell %d)", a / 9, a % 9);
            return UTTT_ERR_ARG;
        }
        s.own[a / 27] |= (uint32_t)pieces[a] << (a % 27);
        s.opp[a / 27] |= (uint32_t)enemy[a] << (a % 27);
    }
    for (int b = 0; b < 9; ++b) {
        if ((uint32_t)main_p[b] > 1u || (uint32_t)main_e[b] > 1u) {
            set_error("main board entries must be 0 or 1 (board %d)", b);
            return UTTT_ERR_ARG;
        }
        s.mains |= ((uint32_t)main_p[b] << b) | ((uint32_t)main_e[b] << (16 + b));
    }
    s.active = active;
    *out = s;
    return UTTT_OK;
}

void uttt_state_to_arrays(const uttt_state_t *s, int32_t pieces[81], int32_t enemy[81], int32_t main_p[9],
                          int32_t main_e[9], int32_t *active) {
    for (int a = 0; a < 81; ++a) {
        if (pieces) pieces[a] = (int32_t)bit_of(s->own, a);
        if (enemy) enemy[a] = (int32_t)bit_of(s->opp, a);
    }
    for (int b = 0; b < 9; ++b) {
        if (main_p) main_p[b] = (int32_t)((s->mains >> b) & 1u);
        if (main_e) main_e[b] = (int32_t)((s->mains >> (16 + b)) & 1u);
    }
    if (active) *active = s->active;
}

int uttt_state_next(const uttt_state_t *s, int32_t action, uttt_state_t *out) {
    if (action < 0 || action > 80) {
        set_error("action must be 0..80 (got %d)", action);
        return UTTT_ERR_ARG;
    }
    *out = next_state(*s, action);
    return UTTT_OK;
}

int uttt_state_legal_actions(const uttt_state_t *s, int32_t out[81]) {
    uint32_t m[3];
    legal_mask(*s, m);
    int n = 0;
    for (int w = 0; w < 3; ++w)
        for (uint32_t bits = m[w]; bits; bits &= bits - 1u) out[n++] = 27 * w + __builtin_ctz(bits);
    return n;
}

int uttt_state_is_lose(const uttt_state_t *s) { return is_lose(*s) ? 1 : 0; }
int uttt_state_is_draw(const uttt_state_t *s) { return (!is_lose(*s) && legal_count(*s) == 0u) ? 1 : 0; }
int uttt_state_is_done(const uttt_state_t *s) { return is_done(*s) ? 1 : 0; }
int uttt_state_is_first_player(const uttt_state_t *s) { return is_first_player(*s) ? 1 : 0; }

void uttt_state_input_hwc(const uttt_state_t *s, float out[243]) {
    uint32_t m[3];
    legal_mask(*s, m);
    for (int a = 0; a < 81; ++a) {
        const int pos = image_index(a);
        out[pos * 3 + 0] = bit_of(s->own, a) ? 1.0f : 0.0f;
        out[pos * 3 + 1] = bit_of(s->opp, a) ? 1.0f : 0.0f;
        out[pos * 3 + 2] = bit_of(m, a) ? 1.0f : 0.0f;
    }
}

int uttt_states_input_hwc(const uttt_state_t *s, int64_t n, float *out) {
    if ((!s || !out) && n > 0) {
        set_error("uttt_states_input_hwc: null pointer");
        return UTTT_ERR_ARG;
    }
    for (int64_t i = 0; i < n; ++i) uttt_state_input_hwc(s + i, out + 243 * i);
    return UTTT_OK;
}

int uttt_state_to_string(const uttt_state_t *s, char *buf, int32_t cap) {
    // Layout of cpp/uttt_game.cpp:194-241 (board rows, main-board status, side, active board).
    const char *ox = is_first_player(*s) ? "ox" : "xo";
    std::string o;
    o.reserve(512);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) {
            for (int i = 0; i < 3; ++i) {
                const int b = r * 3 + i;
                for (int j = 0; j < 3; ++j) {
                    const int a = b * 9 + c * 3 + j;
                    o += bit_of(s->own, a) ? ox[0] : (bit_of(s->opp, a) ? ox[1] : '-');
                    o += ' ';
                }
                if (i < 2) o += "| ";
            }
            o += '\n';
        }
        if (r < 2) o += "---------------------\n";
    }
    o += "\nMain Board Status:\n";
    for (int b = 0; b < 9; ++b) {
        const bool mp = (s->mains >> b) & 1u, me = (s->mains >> (16 + b)) & 1u;
        o += (mp && me) ? 'D' : (mp ? ox[0] : (me ? ox[1] : '.'));
        if (b % 3 == 2) o += '\n';
    }
    o += "Next Player: ";
    o += ox[0];
    o += "\nActive Board: ";
    o += (s->active == -1) ? std::string("Any") : std::to_string(s->active);
    o += '\n';
    const int n = (int)o.size();
    if (!buf || n + 1 > cap) return -(n + 1);
    std::memcpy(buf, o.c_str(), (size_t)n + 1);
    return n;
}

int uttt_boltzman(const float *xs, int32_t n, float temperature, float *out) {
    // cpp/uttt_mcts.cpp:199-216: powf(x, 1/t), sequential f32 sum, divide if sum > 0.
    float sum = 0.0f;
    const float inv = 1.0f / temperature;
    for (int i = 0; i < n; ++i) {
        out[i] = std::pow(xs[i], inv);
        sum += out[i];
    }
    if (sum > 0)
        for (int i = 0; i < n; ++i) out[i] /= sum;
    return n;
}

}  // extern "C"
