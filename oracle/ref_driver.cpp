// oracle/ref_driver.cpp — TEST INFRASTRUCTURE ONLY.
//
// A C-ABI driver around the reference's own C++ hot path, compiled from the
// reference sources where they lie (cpp/uttt_game.cpp, cpp/uttt_mcts.cpp) by
// oracle/Makefile into oracle/_ref/libuttt_ref.so. No reference source is
// copied into this repository; this file only calls the reference API:
//   UTTT::State (cpp/uttt_game.h:11-59), UTTT::pv_mcts_scores and
//   UTTT::boltzman (cpp/uttt_mcts.h:59-68), with an InferenceFunc
//   (cpp/uttt_mcts.h:19) that evaluates every state it is handed with the
//   deterministic hash evaluator (or_hash_eval, oracle/uttt_oracle.c).
//
// Used by tests/golden/make_golden.py (fixtures) and by bench.py's
// cpu_baseline leg (tree-only reference timing). Never by the product.
#include <array>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "uttt_game.h"
#include "uttt_mcts.h"

extern "C" void or_hash_eval(const float *x, float *policy, float *value);

namespace {

using Board = std::array<std::array<int, 9>, 9>;
using Main = std::array<int, 9>;

UTTT::State make_state(const int32_t *pieces81, const int32_t *enemy81, const int32_t *main9,
                       const int32_t *main_e9, int32_t active) {
    Board p{}, e{};
    Main m{}, me{};
    for (int b = 0; b < 9; ++b)
        for (int c = 0; c < 9; ++c) {
            p[b][c] = pieces81[b * 9 + c];
            e[b][c] = enemy81[b * 9 + c];
        }
    for (int i = 0; i < 9; ++i) {
        m[i] = main9[i];
        me[i] = main_e9[i];
    }
    return UTTT::State(p, e, m, me, active);
}

void dump_state(const UTTT::State &s, int32_t *pieces81, int32_t *enemy81, int32_t *main9,
                int32_t *main_e9, int32_t *active) {
    for (int b = 0; b < 9; ++b)
        for (int c = 0; c < 9; ++c) {
            pieces81[b * 9 + c] = s.get_pieces()[b][c];
            enemy81[b * 9 + c] = s.get_enemy_pieces()[b][c];
        }
    for (int i = 0; i < 9; ++i) {
        main9[i] = s.get_main_board_pieces()[i];
        main_e9[i] = s.get_main_board_enemy_pieces()[i];
    }
    *active = s.get_active_board();
}

struct Counters {
    int64_t flushes = 0;
    int64_t evals = 0;
    int64_t unique_per_flush_max = 0;
};

// HWC (pv_mcts_cpp.py:50-53) -> NCHW (pv_mcts_cpp.py:60), then the hash.
void eval_state_hash(const UTTT::State &s, float *policy, float *value) {
    std::vector<float> t = s.to_input_tensor();
    float x[243];
    for (int r = 0; r < 9; ++r)
        for (int c = 0; c < 9; ++c)
            for (int ch = 0; ch < 3; ++ch) x[ch * 81 + r * 9 + c] = t[r * 27 + c * 3 + ch];
    or_hash_eval(x, policy, value);
}

UTTT::InferenceFunc hash_model(Counters *cnt) {
    return [cnt](const std::vector<UTTT::State> &states) {
        std::vector<UTTT::InferenceResult> out;
        out.reserve(states.size());
        cnt->flushes++;
        cnt->evals += (int64_t)states.size();
        // count distinct states in this flush (Appendix A Q3 of SURVEY.md says 1)
        int64_t uniq = 0;
        for (size_t i = 0; i < states.size(); ++i) {
            bool seen = false;
            for (size_t j = 0; j < i && !seen; ++j)
                seen = states[i].get_pieces() == states[j].get_pieces() &&
                       states[i].get_enemy_pieces() == states[j].get_enemy_pieces() &&
                       states[i].get_active_board() == states[j].get_active_board();
            uniq += !seen;
        }
        if (uniq > cnt->unique_per_flush_max) cnt->unique_per_flush_max = uniq;
        for (const auto &s : states) {
            UTTT::InferenceResult r;
            r.policy.resize(81);
            eval_state_hash(s, r.policy.data(), &r.value);
            out.push_back(std::move(r));
        }
        return out;
    };
}

}  // namespace

extern "C" {

int ref_legal_actions(const int32_t *p, const int32_t *e, const int32_t *m, const int32_t *me,
                      int32_t active, int32_t *out) {
    UTTT::State s = make_state(p, e, m, me, active);
    std::vector<int> a = s.legal_actions();
    for (size_t i = 0; i < a.size(); ++i) out[i] = a[i];
    return (int)a.size();
}

// flags: bit0 is_lose, bit1 is_draw, bit2 is_done, bit3 is_first_player
int ref_flags(const int32_t *p, const int32_t *e, const int32_t *m, const int32_t *me, int32_t active) {
    UTTT::State s = make_state(p, e, m, me, active);
    return (s.is_lose() ? 1 : 0) | (s.is_draw() ? 2 : 0) | (s.is_done() ? 4 : 0) |
           (s.is_first_player() ? 8 : 0);
}

void ref_next(const int32_t *p, const int32_t *e, const int32_t *m, const int32_t *me, int32_t active,
              int32_t action, int32_t *op, int32_t *oe, int32_t *om, int32_t *ome, int32_t *oactive) {
    UTTT::State s = make_state(p, e, m, me, active);
    UTTT::State n = s.next(action);
    dump_state(n, op, oe, om, ome, oactive);
}

void ref_tensor(const int32_t *p, const int32_t *e, const int32_t *m, const int32_t *me, int32_t active,
                float *out243) {
    UTTT::State s = make_state(p, e, m, me, active);
    std::vector<float> t = s.to_input_tensor();
    std::memcpy(out243, t.data(), sizeof(float) * 243);
}

int ref_to_string(const int32_t *p, const int32_t *e, const int32_t *m, const int32_t *me,
                  int32_t active, char *buf, int cap) {
    UTTT::State s = make_state(p, e, m, me, active);
    std::string str = s.to_string();
    int n = (int)str.size();
    if (n + 1 > cap) return -n;
    std::memcpy(buf, str.c_str(), (size_t)n + 1);
    return n;
}

// pv_mcts_scores with the hash evaluator. stats (may be NULL): [flushes, evals, max unique/flush]
int ref_search_hash(const int32_t *p, const int32_t *e, const int32_t *m, const int32_t *me,
                    int32_t active, float temperature, int evaluate_count, int batch_size,
                    float *scores_out, int64_t *stats) {
    UTTT::State s = make_state(p, e, m, me, active);
    Counters cnt;
    std::vector<float> sc = UTTT::pv_mcts_scores(hash_model(&cnt), s, temperature, evaluate_count, batch_size);
    for (size_t i = 0; i < sc.size(); ++i) scores_out[i] = sc[i];
    if (stats) {
        stats[0] = cnt.flushes;
        stats[1] = cnt.evals;
        stats[2] = cnt.unique_per_flush_max;
    }
    return (int)sc.size();
}

int ref_boltzman(const float *xs, int n, float temperature, float *out) {
    std::vector<float> v(xs, xs + n);
    std::vector<float> r = UTTT::boltzman(v, temperature);
    for (size_t i = 0; i < r.size(); ++i) out[i] = r[i];
    return (int)r.size();
}

// Tree-only throughput of the reference search (hash evaluator, no NN):
// plays `moves` consecutive searches along a fixed line (the first legal move
// with the highest score each time, restarting from the initial position when
// a game ends). Returns simulations per second on the calling thread.
double ref_bench_tree(int evaluate_count, int batch_size, int moves, int64_t *sims_out) {
    UTTT::State s;
    Counters cnt;
    auto model = hash_model(&cnt);
    int64_t sims = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int mv = 0; mv < moves; ++mv) {
        if (s.is_done()) s = UTTT::State();
        std::vector<float> sc = UTTT::pv_mcts_scores(model, s, 1.0f, evaluate_count, batch_size);
        std::vector<int> legal = s.legal_actions();
        size_t best = 0;
        for (size_t i = 1; i < sc.size(); ++i)
            if (sc[i] > sc[best]) best = i;
        s = s.next(legal[best]);
        sims += evaluate_count;
    }
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (sims_out) *sims_out = sims;
    return (double)sims / dt;
}

}  // extern "C"
