// uttt_cpp_module.cpp — the `uttt_cpp` Python module (drop-in for the
// reference's cpp/python_bindings.cpp:49-107), a thin pybind11 layer over the
// C ABI in include/uttt_engine.h. State is the packed host value type;
// pv_mcts_scores runs the search on the GPU engine (one tree) and calls the
// Python model once per flush (python_bindings.cpp:11-47 contract).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <array>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "uttt_engine.h"

namespace py = pybind11;

namespace {

struct State {
    uttt_state_t s;
    State() { uttt_state_initial(&s); }
    explicit State(const uttt_state_t &v) : s(v) {}
};

[[noreturn]] void raise_engine(int rc) {
    const std::string msg = uttt_last_error();
    if (rc == UTTT_ERR_ARG) throw py::value_error(msg);
    throw std::runtime_error(msg);
}

void check(int rc) {
    if (rc != UTTT_OK) raise_engine(rc);
}

template <size_t N>
void seq_to_ints(const py::handle &obj, int32_t *out, const char *what) {
    py::sequence seq = py::reinterpret_borrow<py::sequence>(obj);
    if ((size_t)py::len(seq) != N) throw py::type_error(std::string(what) + ": expected " + std::to_string(N) + " entries");
    for (size_t i = 0; i < N; ++i) out[i] = seq[i].cast<int32_t>();
}

void board_to_ints(const py::handle &obj, int32_t *out, const char *what) {
    py::sequence rows = py::reinterpret_borrow<py::sequence>(obj);
    if (py::len(rows) != 9) throw py::type_error(std::string(what) + ": expected 9 boards of 9 cells");
    for (int b = 0; b < 9; ++b) seq_to_ints<9>(rows[b], out + 9 * b, what);
}

py::list board_list(const int32_t *v) {
    py::list rows;
    for (int b = 0; b < 9; ++b) {
        py::list r;
        for (int c = 0; c < 9; ++c) r.append(v[9 * b + c]);
        rows.append(r);
    }
    return rows;
}

// One cached single-tree engine for pv_mcts_scores (the GIL serialises use,
// as in the reference where the search holds the GIL throughout).
struct SearchEngine {
    uttt_engine_t *eng = nullptr;
    int max_sims = 0;
    ~SearchEngine() {
        if (eng) uttt_engine_destroy(eng);
    }
    uttt_engine_t *get(int sims) {
        // The engine's 16-byte node record holds N, k and the first-child index in 16 / 12 / 20 bits
        // (engine.hip, struct Pool): a tree of at most 4095 simulations. The reference has no such
        // bound (uttt_mcts.cpp heap nodes); every caller in the reference uses 50 (self-play, arena)
        // or 10 (test_cpp_mcts.py). Refused here, before any device work, with the reason.
        if (sims > UTTT_MAX_SIMS)
            throw py::value_error("pv_mcts_scores: evaluate_count " + std::to_string(sims) + " exceeds " +
                                  std::to_string(UTTT_MAX_SIMS) +
                                  ", the most simulations this engine's 16-byte node records hold per search "
                                  "(INTEGRATION.md, limits)");
        if (!eng || sims > max_sims) {
            if (eng) uttt_engine_destroy(eng);
            eng = nullptr;
            const int cap = sims > 400 ? sims : 400;
            check(uttt_engine_create(-1, 1, cap, &eng));
            max_sims = cap;
        }
        return eng;
    }
};

SearchEngine &search_engine() {
    static SearchEngine *se = new SearchEngine();  // leaked on purpose: no HIP calls at interpreter exit
    return *se;
}

// Read one (policy, value) result tuple as python_bindings.cpp:24-43 does.
void read_result(const py::handle &item, float *policy81, float *value) {
    py::tuple tup = py::reinterpret_borrow<py::object>(item).cast<py::tuple>();
    py::object pol = tup[0];
    if (py::isinstance<py::array>(pol)) {
        auto arr = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(pol);
        if (!arr) throw py::type_error("policy must be convertible to float32");
        const int n = (int)std::min<py::ssize_t>(arr.size(), 81);
        std::memcpy(policy81, arr.data(), (size_t)n * sizeof(float));
        for (int a = n; a < 81; ++a) policy81[a] = 0.0f;  // uttt_mcts.cpp:149
    } else {
        const std::vector<float> p = pol.cast<std::vector<float>>();
        for (int a = 0; a < 81; ++a) policy81[a] = a < (int)p.size() ? p[a] : 0.0f;
    }
    *value = tup[1].cast<float>();
}

py::list pv_mcts_scores(py::object model, const State &state, float temperature, int evaluate_count, int batch_size,
                        bool dedup) {
    if (evaluate_count <= 0) {
        // the reference loop body never runs: every root child keeps n == 0
        std::vector<int32_t> legal(81);
        const int L = uttt_state_legal_actions(&state.s, legal.data());
        std::vector<float> sc(L, 0.0f), out(L);
        if (temperature == 0.0f) {
            if (L) sc[0] = 1.0f;
            out = sc;
        } else {
            uttt_boltzman(sc.data(), L, temperature, out.data());
        }
        return py::cast(out);
    }
    uttt_engine_t *eng = search_engine().get(evaluate_count);
    // round 6: the whole search as one resident wave (uttt_search1_*: no launch per flush, the scores
    // stored by the wave at the end); UTTT_SEARCH1=0 keeps the launch per flush of round 5
    static const bool resident = [] {
        const char *v = getenv("UTTT_SEARCH1");
        return !(v && v[0] == '0');
    }();
    if (resident) check(uttt_search1_begin(eng, &state.s, evaluate_count, batch_size, UTTT_SEMANTICS_CPP, temperature));
    else check(uttt_search_begin(eng, &state.s, 1, evaluate_count, batch_size));
    // per flush: the round's leaf and its copies k come back through pinned host memory the scan writes
    // (uttt_search_select_host), the results go to pinned memory k_apply reads (uttt_search_apply_host): no
    // copy operation and no stream synchronisation per flush besides the model's own
    std::vector<float> pol, val;
    for (;;) {
        int32_t n = 0, k = 0;
        uttt_state_t leaf;
        if (resident) check(uttt_search1_next(eng, &leaf, &k, &n));
        else check(uttt_search_select_host(eng, &leaf, &k, &n));
        if (n == 0) break;
        const int copies = dedup ? 1 : k;
        py::list batch;
        for (int i = 0; i < copies; ++i) batch.append(py::cast(State(leaf)));
        py::object result = model(batch);
        pol.assign((size_t)copies * 81, 0.0f);
        val.assign((size_t)copies, 0.0f);
        int got = 0;
        for (auto item : result) {
            if (got >= copies) break;
            read_result(item, pol.data() + 81 * got, val.data() + got);
            ++got;
        }
        if (got < copies)
            throw std::runtime_error("model returned " + std::to_string(got) + " results for " + std::to_string(copies) +
                                     " states");
        if (resident) check(uttt_search1_apply(eng, pol.data(), 81, val.data(), copies));
        else check(uttt_search_apply_host(eng, pol.data(), 81, val.data(), copies));
    }
    float scores[81];
    int32_t L = 0;
    if (resident) check(uttt_search1_scores(eng, scores, &L));
    else check(uttt_search_scores(eng, temperature, scores, &L));
    return py::cast(std::vector<float>(scores, scores + L));
}

}  // namespace

PYBIND11_MODULE(_uttt_cpp, m) {
    m.doc() = "Ultimate Tic-Tac-Toe rules + MI355X (gfx950) PV-MCTS engine; drop-in for the reference uttt_cpp";
    m.attr("__version__") = uttt_version();
    m.attr("backend") = "hip-gfx950";

    py::class_<State>(m, "State")
        .def(py::init<>())
        .def(py::init([](py::object pieces, py::object enemy, py::object main_p, py::object main_e, int active) {
                 int32_t p[81], e[81], mp[9], me[9];
                 board_to_ints(pieces, p, "pieces");
                 board_to_ints(enemy, e, "enemy_pieces");
                 seq_to_ints<9>(main_p, mp, "main_board_pieces");
                 seq_to_ints<9>(main_e, me, "main_board_enemy_pieces");
                 State s;
                 check(uttt_state_from_arrays(p, e, mp, me, active, &s.s));
                 return s;
             }),
             py::arg("pieces"), py::arg("enemy_pieces"), py::arg("main_board_pieces"),
             py::arg("main_board_enemy_pieces"), py::arg("active_board"))
        .def("is_lose", [](const State &s) { return uttt_state_is_lose(&s.s) != 0; })
        .def("is_draw", [](const State &s) { return uttt_state_is_draw(&s.s) != 0; })
        .def("is_done", [](const State &s) { return uttt_state_is_done(&s.s) != 0; })
        .def("is_first_player", [](const State &s) { return uttt_state_is_first_player(&s.s) != 0; })
        .def("next",
             [](const State &s, int action) {
                 State n;
                 check(uttt_state_next(&s.s, action, &n.s));
                 return n;
             })
        .def("legal_actions",
             [](const State &s) {
                 int32_t out[81];
                 const int n = uttt_state_legal_actions(&s.s, out);
                 return std::vector<int>(out, out + n);
             })
        .def("to_string",
             [](const State &s) {
                 char buf[1024];
                 const int n = uttt_state_to_string(&s.s, buf, sizeof(buf));
                 if (n < 0) throw std::runtime_error("to_string buffer");
                 return std::string(buf, (size_t)n);
             })
        .def("__str__",
             [](const State &s) {
                 char buf[1024];
                 const int n = uttt_state_to_string(&s.s, buf, sizeof(buf));
                 if (n < 0) throw std::runtime_error("to_string buffer");
                 return std::string(buf, (size_t)n);
             })
        .def("to_input_tensor",
             [](const State &s) {
                 std::vector<float> t(243);
                 uttt_state_input_hwc(&s.s, t.data());
                 return t;
             })
        .def_property_readonly("pieces",
                               [](const State &s) {
                                   int32_t p[81];
                                   uttt_state_to_arrays(&s.s, p, nullptr, nullptr, nullptr, nullptr);
                                   return board_list(p);
                               })
        .def_property_readonly("enemy_pieces",
                               [](const State &s) {
                                   int32_t e[81];
                                   uttt_state_to_arrays(&s.s, nullptr, e, nullptr, nullptr, nullptr);
                                   return board_list(e);
                               })
        .def_property_readonly("main_board_pieces",
                               [](const State &s) {
                                   int32_t mp[9];
                                   uttt_state_to_arrays(&s.s, nullptr, nullptr, mp, nullptr, nullptr);
                                   return std::vector<int>(mp, mp + 9);
                               })
        .def_property_readonly("main_board_enemy_pieces",
                               [](const State &s) {
                                   int32_t me[9];
                                   uttt_state_to_arrays(&s.s, nullptr, nullptr, nullptr, me, nullptr);
                                   return std::vector<int>(me, me + 9);
                               })
        .def_property_readonly("active_board", [](const State &s) { return (int)s.s.active; })
        // extensions (not in the reference): the packed 32-byte value, for batching
        .def_property_readonly("packed",
                               [](const State &s) {
                                   return py::bytes(reinterpret_cast<const char *>(&s.s), sizeof(uttt_state_t));
                               })
        .def_static("from_packed", [](py::bytes b) {
            std::string raw = b;
            if (raw.size() != sizeof(uttt_state_t)) throw py::value_error("packed state must be 32 bytes");
            State s;
            std::memcpy(&s.s, raw.data(), sizeof(uttt_state_t));
            return s;
        });

    struct InferenceResult {
        std::vector<float> policy;
        float value = 0.0f;
    };
    py::class_<InferenceResult>(m, "InferenceResult")
        .def(py::init<>())
        .def_readwrite("policy", &InferenceResult::policy)
        .def_readwrite("value", &InferenceResult::value);

    m.def("pv_mcts_scores", &pv_mcts_scores, py::arg("model"), py::arg("state"), py::arg("temperature") = 0.0f,
          py::arg("evaluate_count") = 50, py::arg("batch_size") = 8, py::arg("dedup") = false,
          "Run MCTS (on the MI355X engine) and return score distribution over legal actions. The model gets the k "
          "identical queued states of each flush, as the reference's module passes them (python_bindings.cpp:11-47); "
          "dedup=True hands it one state and applies its result k times (same scores for a deterministic model)");
    m.def(
        "boltzman",
        [](const std::vector<float> &xs, float temperature) {
            std::vector<float> out(xs.size());
            uttt_boltzman(xs.data(), (int32_t)xs.size(), temperature, out.data());
            return out;
        },
        py::arg("xs"), py::arg("temperature"), "Apply Boltzmann distribution");
    m.def(
        "_search1_time_split",
        [] {
            int32_t t[3] = {0, 0, 0};
            uttt_engine_t *eng = search_engine().eng;
            if (eng) check(uttt_search1_time_split(eng, t));
            return std::vector<double>{t[0] * 1e-5, t[1] * 1e-5, t[2] * 1e-5};
        },
        "Diagnostics: the last resident search's device time in ms (descents, applies, waits for the host)");
}
