/*
 * oracle/uttt_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * A plain-C restatement of the reference hot path, used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg — and by nothing
 * else. The product (ultimate-tictactoe-alphazero_amd/) never links, loads or
 * calls this file; it runs the HIP kernels or fails.
 *
 * Restated from (all paths under the reference checkout):
 *   rules   cpp/uttt_game.cpp   (State, check_win, next, legal_actions, tensor)
 *   search  cpp/uttt_mcts.cpp   (Node, search_leaf, expand, backprop, PUCT, pv_mcts_scores, boltzman)
 *   driver  self_play_cpp.py    (play: f64 renormalisation, np.random.choice, value back-fill)
 *   numpy   legacy RandomState  (MT19937 seeding/tempering, random_sample, choice(p=...)),
 *           pairwise float64 summation of np.add.reduce (PW_BLOCKSIZE 128, 8 accumulators).
 *
 * Deliberately structured like the reference (heap nodes that each hold a full
 * State copy, children appended, every queued copy evaluated separately) so it
 * is an independent check of the engine's de-duplicated, bitboard, SoA design.
 *
 * Pinned by: the tests/golden fixtures, produced by tests/golden/make_golden.py from the
 * reference compiled from its own sources (oracle/Makefile -> oracle/_ref/) and
 * from the reference Python driver (self_play_cpp.play) imported in the build
 * container. See tests/test_oracle.py.
 *
 * Build: gcc -O2 -std=c11 -ffp-contract=off -fPIC -shared (no FMA contraction,
 * x86-64 SSE arithmetic: the same IEEE single/double rounding as the reference).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* State (cpp/uttt_game.h:11-59)                                              */
/* ------------------------------------------------------------------------- */
typedef struct or_state {
    int32_t pieces[9][9];   /* side to move, [board][cell]           */
    int32_t enemy[9][9];    /* opponent                              */
    int32_t main_p[9];      /* main_board_pieces_                    */
    int32_t main_e[9];      /* main_board_enemy_pieces_              */
    int32_t active;         /* -1 = any, 0..8                        */
} or_state;

void or_state_initial(or_state *s) { /* uttt_game.cpp:9-21 */
    memset(s, 0, sizeof(*s));
    s->active = -1;
}

/* uttt_game.cpp:35-61: is_comp(x, y, dx, dy) walks 3 cells at x + 3y; any 0 fails. */
static int or_is_comp(const int32_t *b, int x, int y, int dx, int dy) {
    for (int k = 0; k < 3; ++k) {
        if (y < 0 || y > 2 || x < 0 || x > 2 || b[x + y * 3] == 0) return 0;
        x += dx;
        y += dy;
    }
    return 1;
}

int or_check_win(const int32_t *b) {
    if (or_is_comp(b, 0, 0, 1, 1) || or_is_comp(b, 0, 2, 1, -1)) return 1;
    for (int i = 0; i < 3; ++i)
        if (or_is_comp(b, 0, i, 1, 0) || or_is_comp(b, i, 0, 0, 1)) return 1;
    return 0;
}

/* uttt_game.cpp:77-79: only the OPPONENT's main board is inspected (Q8). */
int or_is_lose(const or_state *s) { return or_check_win(s->main_e); }

/* uttt_game.cpp:148-191: ascending board, then ascending cell. */
int or_legal_actions(const or_state *s, int32_t *out) {
    int n = 0;
    if (or_is_lose(s)) return 0;
    int cand[9], nc = 0;
    if (s->active == -1) {
        for (int i = 0; i < 9; ++i)
            if (s->main_p[i] == 0 && s->main_e[i] == 0) cand[nc++] = i;
    } else {
        int a = s->active;
        if (s->main_p[a] == 0 && s->main_e[a] == 0) {
            cand[nc++] = a;
        } else {
            for (int i = 0; i < 9; ++i)
                if (s->main_p[i] == 0 && s->main_e[i] == 0) cand[nc++] = i;
        }
    }
    for (int bi = 0; bi < nc; ++bi) {
        int b = cand[bi];
        for (int c = 0; c < 9; ++c)
            if (s->pieces[b][c] == 0 && s->enemy[b][c] == 0) out[n++] = b * 9 + c;
    }
    return n;
}

/* uttt_game.cpp:82-89 */
int or_is_draw(const or_state *s) {
    int32_t tmp[81];
    return !or_is_lose(s) && or_legal_actions(s, tmp) == 0;
}
int or_is_done(const or_state *s) { return or_is_lose(s) || or_is_draw(s); }

/* uttt_game.cpp:64-74, 92-94: counts cells equal to 1. */
static int or_piece_count(const int32_t p[9][9]) {
    int c = 0;
    for (int b = 0; b < 9; ++b)
        for (int j = 0; j < 9; ++j) c += (p[b][j] == 1);
    return c;
}
int or_is_first_player(const or_state *s) {
    return or_piece_count(s->pieces) == or_piece_count(s->enemy);
}

/* uttt_game.cpp:97-145: swap sides, mover's stone lands in the new enemy board;
 * small win -> new enemy main flag; full small board -> BOTH flags (Q7);
 * next active = cell unless that board is closed. */
void or_next(const or_state *s, int action, or_state *o) {
    int b = action / 9, c = action % 9;
    or_state n;
    memcpy(n.pieces, s->enemy, sizeof(n.pieces));
    memcpy(n.enemy, s->pieces, sizeof(n.enemy));
    memcpy(n.main_p, s->main_e, sizeof(n.main_p));
    memcpy(n.main_e, s->main_p, sizeof(n.main_e));
    n.enemy[b][c] = 1;
    if (or_check_win(n.enemy[b])) {
        n.main_e[b] = 1;
    } else {
        int full = 1;
        for (int j = 0; j < 9; ++j)
            if (n.pieces[b][j] == 0 && n.enemy[b][j] == 0) { full = 0; break; }
        if (full) { n.main_p[b] = 1; n.main_e[b] = 1; }
    }
    int na = c;
    if (n.main_p[na] == 1 || n.main_e[na] == 1) na = -1;
    n.active = na;
    *o = n;
}

/* uttt_game.cpp:244-280: HWC (9,9,3); cell (b,c) -> R=(b/3)*3+c/3, C=(b%3)*3+c%3. */
void or_tensor_hwc(const or_state *s, float *t) {
    int32_t leg[81];
    int nl = or_legal_actions(s, leg);
    for (int i = 0; i < 243; ++i) t[i] = 0.0f;
    for (int b = 0; b < 9; ++b)
        for (int c = 0; c < 9; ++c) {
            int R = (b / 3) * 3 + c / 3, C = (b % 3) * 3 + c % 3;
            if (s->pieces[b][c] == 1) t[R * 27 + C * 3 + 0] = 1.0f;
            if (s->enemy[b][c] == 1) t[R * 27 + C * 3 + 1] = 1.0f;
        }
    for (int i = 0; i < nl; ++i) {
        int b = leg[i] / 9, c = leg[i] % 9;
        int R = (b / 3) * 3 + c / 3, C = (b % 3) * 3 + c % 3;
        t[R * 27 + C * 3 + 2] = 1.0f;
    }
}

/* The NCHW view the glue hands the network (pv_mcts_cpp.py:50-60). */
void or_tensor_nchw(const or_state *s, float *x) {
    float t[243];
    or_tensor_hwc(s, t);
    for (int r = 0; r < 9; ++r)
        for (int c = 0; c < 9; ++c)
            for (int ch = 0; ch < 3; ++ch) x[ch * 81 + r * 9 + c] = t[r * 27 + c * 3 + ch];
}

/* ------------------------------------------------------------------------- */
/* Deterministic hash evaluator (test evaluator; spec in DESIGN.md §Hash).    */
/* Input: the NCHW tensor (3,9,9). Bit j = ch*81 + R*9 + C set iff x[j] != 0. */
/* ------------------------------------------------------------------------- */
static uint64_t or_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* salt != 0 gives a different deterministic player: h = mix64(h ^ salt) */
void or_hash_eval_salted(const float *x, float *policy, float *value, uint64_t salt) {
    uint64_t w[4] = {0, 0, 0, 0};
    for (int j = 0; j < 243; ++j)
        if (x[j] != 0.0f) w[j >> 6] |= 1ULL << (j & 63);
    uint64_t h = 0x9E3779B97F4A7C15ULL;
    for (int i = 0; i < 4; ++i) h = or_mix64(h ^ w[i]);
    if (salt) h = or_mix64(h ^ salt);
    uint32_t mode = (uint32_t)((h >> 8) & 15u);
    for (int a = 0; a < 81; ++a) {
        uint64_t r = or_mix64(h + (uint64_t)(a + 1) * 0x9E3779B97F4A7C15ULL);
        float p = (float)(uint32_t)(r >> 40) * (1.0f / 16777216.0f);
        if (mode == 0) p = 0.0f;                         /* exercises the sum<=0 path  */
        else if (mode == 1) p = p * 0x1p-140f;           /* subnormal priors (FTZ trap) */
        else if (mode == 2 && (a & 3)) p = 0.0f;         /* sparse priors              */
        policy[a] = p;
    }
    uint64_t rv = or_mix64(h ^ 0xD6E8FEB86659FD93ULL);
    *value = (float)((int32_t)(rv % 2001ULL) - 1000) / 1000.0f;
}

void or_hash_eval(const float *x, float *policy, float *value) { or_hash_eval_salted(x, policy, value, 0ULL); }

/* ------------------------------------------------------------------------- */
/* PV-MCTS (cpp/uttt_mcts.cpp)                                                */
/* ------------------------------------------------------------------------- */
typedef void (*or_eval_fn)(const float *x_nchw, float *policy81, float *value, void *ctx);

typedef struct or_node {
    or_state s;
    float p, w;
    int n;
    struct or_node **ch;
    int nch, cap;
} or_node;

typedef struct or_search_stats {
    int32_t flushes;      /* model() calls                                   */
    int32_t evals;        /* states handed to the model (with duplicates)    */
    int32_t terminal;     /* simulations that ended on a terminal node       */
    int32_t max_depth;    /* longest path (edges)                            */
    int32_t nodes;        /* nodes allocated, root included                  */
    int32_t max_children; /* widest child list                               */
} or_search_stats;

static or_node *or_node_new(const or_state *s, float p) { /* uttt_mcts.cpp:10-12 */
    or_node *n = (or_node *)calloc(1, sizeof(or_node));
    n->s = *s;
    n->p = p;
    return n;
}

static void or_node_free(or_node *n) {
    for (int i = 0; i < n->nch; ++i) or_node_free(n->ch[i]);
    free(n->ch);
    free(n);
}

/* uttt_mcts.cpp:35-44: APPENDS children (never clears; Q5). */
static void or_expand(or_node *nd, const float *pol, int npol, or_search_stats *st) {
    int32_t leg[81];
    int nl = or_legal_actions(&nd->s, leg);
    for (int i = 0; i < nl; ++i) {
        float p = (i < npol) ? pol[i] : 0.0f;
        or_state ns;
        or_next(&nd->s, leg[i], &ns);
        if (nd->nch == nd->cap) {
            nd->cap = nd->cap ? nd->cap * 2 : 16;
            nd->ch = (or_node **)realloc(nd->ch, sizeof(or_node *) * (size_t)nd->cap);
        }
        nd->ch[nd->nch++] = or_node_new(&ns, p);
        st->nodes++;
    }
    if (nd->nch > st->max_children) st->max_children = nd->nch;
}

/* uttt_mcts.cpp:47-54 */
static void or_backprop(or_node **path, int len, float value) {
    for (int i = len - 1; i >= 0; --i) {
        path[i]->w += value;
        path[i]->n += 1;
        value = -value;
    }
}

/* uttt_mcts.cpp:57-81: f32 PUCT, c=1, strict '>' from -1e9f (first index wins). */
static or_node *or_next_child(or_node *nd) {
    const float C_PUCT = 1.0f;
    int total = 0;
    for (int i = 0; i < nd->nch; ++i) total += nd->ch[i]->n;
    float sq = sqrtf((float)total);
    float best = -1e9f;
    or_node *bc = NULL;
    for (int i = 0; i < nd->nch; ++i) {
        or_node *c = nd->ch[i];
        float q = (c->n > 0) ? (-c->w / c->n) : 0.0f;
        float u = C_PUCT * c->p * sq / (1 + c->n);
        float pucb = q + u;
        if (pucb > best) { best = pucb; bc = c; }
    }
    return bc;
}

/* uttt_mcts.cpp:15-32: terminal -> value -(is_lose ? -1 : 0) (sign inverted, Q4). */
static or_node *or_search_leaf(or_node *nd, or_node **path, int *len, float *value) {
    for (;;) {
        path[(*len)++] = nd;
        if (or_is_done(&nd->s)) {
            float v = or_is_lose(&nd->s) ? -1.0f : 0.0f;
            *value = -v;
            return nd;
        }
        if (nd->nch == 0) { *value = 0.0f; return nd; }
        nd = or_next_child(nd);
    }
}

/* uttt_mcts.cpp:199-216 */
int or_boltzman(const float *xs, int n, float temperature, float *out) {
    float sum = 0.0f;
    for (int i = 0; i < n; ++i) {
        out[i] = powf(xs[i], 1.0f / temperature);
        sum += out[i];
    }
    if (sum > 0)
        for (int i = 0; i < n; ++i) out[i] /= sum;
    return n;
}

#define OR_MAX_PATH 512

/* uttt_mcts.cpp:84-196. Returns |legal| (scores length); visits_out gets the
 * root children's visit counts (may be NULL). Every queued copy is evaluated
 * separately, exactly as the reference batch is. */
int or_pv_mcts_scores(const or_state *root_s, float temperature, int evaluate_count, int batch_size,
                      or_eval_fn eval, void *ctx, float *scores_out, int32_t *visits_out,
                      or_search_stats *st_out) {
    or_search_stats st;
    memset(&st, 0, sizeof(st));
    int32_t leg[81];
    int nl = or_legal_actions(root_s, leg);
    if (nl == 0) { if (st_out) *st_out = st; return 0; }
    or_node *root = or_node_new(root_s, 0.0f);
    st.nodes = 1;
    float up[81];
    float uniform = 1.0f / (float)nl;
    for (int i = 0; i < nl; ++i) up[i] = uniform;
    or_expand(root, up, nl, &st);

    int qcap = 64, qn = 0;
    or_node **qleaf = (or_node **)malloc(sizeof(or_node *) * (size_t)qcap);
    or_node ***qpath = (or_node ***)malloc(sizeof(or_node **) * (size_t)qcap);
    int *qlen = (int *)malloc(sizeof(int) * (size_t)qcap);
    or_node *path[OR_MAX_PATH];

    for (int i = 0; i < evaluate_count; ++i) {
        int len = 0;
        float value;
        or_node *leaf = or_search_leaf(root, path, &len, &value);
        if (len - 1 > st.max_depth) st.max_depth = len - 1;
        if (or_is_done(&leaf->s)) { /* :115-118 */
            or_backprop(path, len, value);
            st.terminal++;
            continue;
        }
        if (leaf->n == 0 && leaf->nch == 0) { /* :121-124 */
            if (qn == qcap) {
                qcap *= 2;
                qleaf = (or_node **)realloc(qleaf, sizeof(or_node *) * (size_t)qcap);
                qpath = (or_node ***)realloc(qpath, sizeof(or_node **) * (size_t)qcap);
                qlen = (int *)realloc(qlen, sizeof(int) * (size_t)qcap);
            }
            qleaf[qn] = leaf;
            qpath[qn] = (or_node **)malloc(sizeof(or_node *) * (size_t)len);
            memcpy(qpath[qn], path, sizeof(or_node *) * (size_t)len);
            qlen[qn] = len;
            qn++;
        }
        if (qn >= batch_size || i == evaluate_count - 1) { /* :127 */
            if (qn > 0) {
                st.flushes++;
                for (int j = 0; j < qn; ++j) {
                    or_node *lf = qleaf[j];
                    float x[243], pol[81], v;
                    or_tensor_nchw(&lf->s, x);
                    eval(x, pol, &v, ctx);
                    st.evals++;
                    int32_t ll[81];
                    int nll = or_legal_actions(&lf->s, ll);
                    float lp[81];
                    float psum = 0.0f;
                    for (int a = 0; a < nll; ++a) { /* :144-152 sequential f32 sum */
                        lp[a] = pol[ll[a]];
                        psum += lp[a];
                    }
                    if (psum > 0) {
                        for (int a = 0; a < nll; ++a) lp[a] /= psum;
                    } else {
                        float un = nll ? 1.0f / (float)nll : 0.0f;
                        for (int a = 0; a < nll; ++a) lp[a] = un;
                    }
                    or_expand(lf, lp, nll, &st);
                    or_backprop(qpath[j], qlen[j], v);
                    free(qpath[j]);
                }
                qn = 0;
            }
        }
    }
    float sc[81];
    for (int i = 0; i < root->nch; ++i) {
        sc[i] = (float)root->ch[i]->n;
        if (visits_out) visits_out[i] = root->ch[i]->n;
    }
    if (temperature == 0.0f) { /* :183-189 first max */
        int mi = 0;
        for (int i = 1; i < root->nch; ++i)
            if (sc[i] > sc[mi]) mi = i;
        for (int i = 0; i < root->nch; ++i) scores_out[i] = 0.0f;
        scores_out[mi] = 1.0f;
    } else {
        or_boltzman(sc, root->nch, temperature, scores_out);
    }
    int nout = root->nch;
    free(qleaf);
    free(qpath);
    free(qlen);
    or_node_free(root);
    if (st_out) *st_out = st;
    return nout;
}

void or_eval_hash_cb(const float *x, float *policy, float *value, void *ctx) {
    (void)ctx;
    or_hash_eval(x, policy, value);
}

int or_pv_mcts_scores_hash(const or_state *root, float temperature, int evaluate_count, int batch_size,
                           float *scores_out, int32_t *visits_out, or_search_stats *st) {
    return or_pv_mcts_scores(root, temperature, evaluate_count, batch_size, or_eval_hash_cb, NULL,
                             scores_out, visits_out, st);
}

/* ------------------------------------------------------------------------- */
/* numpy legacy RandomState (MT19937) and the float64 reductions it relies on */
/* ------------------------------------------------------------------------- */
typedef struct or_mt { uint32_t key[624]; int32_t pos; } or_mt;

/* RandomState(seed) for an integer seed == mt19937 init_genrand. */
void or_mt_seed(or_mt *m, uint32_t seed) {
    m->key[0] = seed;
    for (int i = 1; i < 624; ++i)
        m->key[i] = 1812433253u * (m->key[i - 1] ^ (m->key[i - 1] >> 30)) + (uint32_t)i;
    m->pos = 624;
}

static void or_mt_twist(or_mt *m) {
    for (int i = 0; i < 624; ++i) {
        uint32_t y = (m->key[i] & 0x80000000u) | (m->key[(i + 1) % 624] & 0x7fffffffu);
        uint32_t v = m->key[(i + 397) % 624] ^ (y >> 1);
        if (y & 1u) v ^= 0x9908b0dfu;
        m->key[i] = v;
    }
    m->pos = 0;
}

uint32_t or_mt_next32(or_mt *m) {
    if (m->pos >= 624) or_mt_twist(m);
    uint32_t y = m->key[m->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* legacy random_sample(): 53-bit double from two draws. */
double or_mt_double(or_mt *m) {
    uint32_t a = or_mt_next32(m) >> 5, b = or_mt_next32(m) >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

/* np.add.reduce over a contiguous float64 vector: pairwise, 8 accumulators,
 * blocks of <= 128 elements. */
double or_np_pairwise_sum(const double *a, int64_t n) {
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return or_np_pairwise_sum(a, n2) + or_np_pairwise_sum(a + n2, n - n2);
    }
}

/* RandomState.choice(range(n), p=p) with size=None: cdf = cumsum(p);
 * cdf /= cdf[-1]; searchsorted(cdf, random_sample(), 'right'). */
int or_np_choice(or_mt *m, const double *p, int n) {
    double cdf[128];
    double acc = 0.0;
    for (int i = 0; i < n; ++i) { acc += p[i]; cdf[i] = acc; }
    double last = cdf[n - 1];
    for (int i = 0; i < n; ++i) cdf[i] /= last;
    double u = or_mt_double(m);
    int lo = 0;
    while (lo < n && cdf[lo] <= u) ++lo;
    return lo;
}

/* self_play_cpp.py:74-86 for one position: scores (f32, |legal|) -> float64
 * policy over legal moves, renormalised with np.sum; returns the index into
 * legal of the sampled move. */
int or_policy_and_sample(or_mt *m, const float *scores, int n, double *pol) {
    for (int i = 0; i < n; ++i) pol[i] = (double)scores[i];
    double s = or_np_pairwise_sum(pol, n);
    if (s == 0.0) {
        for (int i = 0; i < n; ++i) pol[i] = 1.0 / (double)n;
    } else {
        for (int i = 0; i < n; ++i) pol[i] = pol[i] / s;
    }
    return or_np_choice(m, pol, n);
}

/* self_play_cpp.py:34-101, one game with RandomState(seed) standing in for the
 * global numpy RNG. Outputs per ply: HWC input (243 f32), policy (81 f64),
 * action, value (Q9: ply 0 gets the final value, then alternating). Returns
 * the number of plies (<= max_plies) or -1 on overflow. */
int or_self_play_game(uint32_t seed, float temperature, int evaluate_count, int batch_size,
                      or_eval_fn eval, void *ctx, int max_plies,
                      float *tensors_out, double *policies_out, int32_t *actions_out,
                      int32_t *values_out) {
    or_mt *m = (or_mt *)malloc(sizeof(or_mt));
    or_mt_seed(m, seed);
    or_state s;
    or_state_initial(&s);
    int ply = 0;
    while (!or_is_done(&s)) {
        if (ply >= max_plies) { free(m); return -1; }
        or_tensor_hwc(&s, tensors_out + (size_t)ply * 243);
        float sc[81];
        int32_t leg[81];
        int ns = or_pv_mcts_scores(&s, temperature, evaluate_count, batch_size, eval, ctx, sc, NULL, NULL);
        int nl = or_legal_actions(&s, leg);
        if (ns != nl) { free(m); return -2; }
        double pl[81];
        int idx = or_policy_and_sample(m, sc, nl, pl);
        double *pol = policies_out + (size_t)ply * 81;
        for (int a = 0; a < 81; ++a) pol[a] = 0.0;
        for (int i = 0; i < nl; ++i) pol[leg[i]] = pl[i];
        actions_out[ply] = leg[idx];
        or_state nx;
        or_next(&s, leg[idx], &nx);
        s = nx;
        ply++;
    }
    int v = or_is_lose(&s) ? -1 : 0;
    for (int i = 0; i < ply; ++i) { values_out[i] = v; v = -v; }
    free(m);
    return ply;
}

int or_self_play_game_hash(uint32_t seed, float temperature, int evaluate_count, int batch_size,
                           int max_plies, float *tensors_out, double *policies_out,
                           int32_t *actions_out, int32_t *values_out) {
    return or_self_play_game(seed, temperature, evaluate_count, batch_size, or_eval_hash_cb, NULL,
                             max_plies, tensors_out, policies_out, actions_out, values_out);
}

/* ------------------------------------------------------------------------- */
/* Python PV-MCTS (pv_mcts.py) — the arena path (evaluate_network.py).        */
/* SURVEY Appendix B. Scalar arithmetic follows NumPy 2 promotion (NEP 50:    */
/* Python scalars are "weak"), the numpy of this image and of the fixtures:   */
/*  * priors: policy[legal] (f32) / np.sum (f32 pairwise) (pv_mcts.py:46-56); */
/*    all-zero -> np.ones(float)/L, i.e. float64 priors for that expansion;   */
/*  * w is an int until the first network value (np.float32) is added;        */
/*  * PUCT (:120-130): f32 ops with sqrt(t) in double, or float64 where the   */
/*    prior is float64; np.argmax = first maximum (a NaN counts as maximum);  */
/*  * root not pre-expanded, expand REPLACES the children (:104-108), queue   */
/*    test n == 0 (:150); boltzman in Python floats (:190-192).               */
/* ------------------------------------------------------------------------- */
typedef struct or_pnode {
    or_state s;
    float p;          /* prior (f32) unless p64 */
    int p64;          /* prior is the float64 uniform 1/nsib */
    int nsib;         /* |legal| of the parent (for p64) */
    float w;          /* exact for int-typed w too (|w| small) */
    int w_f32;        /* w has become np.float32 */
    int n;
    struct or_pnode **ch;
    int nch;          /* -1: child_nodes is None */
} or_pnode;

static or_pnode *or_pnode_new(const or_state *s) {
    or_pnode *n = (or_pnode *)calloc(1, sizeof(or_pnode));
    n->s = *s;
    n->nch = -1;
    return n;
}

static void or_pnode_free(or_pnode *n) {
    for (int i = 0; i < n->nch; ++i) or_pnode_free(n->ch[i]);
    free(n->ch);
    free(n);
}

/* np.add.reduce over a contiguous float32 array (pairwise, float32 accumulators) */
float or_np_pairwise_sum_f32(const float *a, int64_t n) {
    if (n < 8) {
        float r = 0.0f;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    } else if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return or_np_pairwise_sum_f32(a, n2) + or_np_pairwise_sum_f32(a + n2, n - n2);
    }
}

/* predict_batch's per-state post-processing (pv_mcts.py:46-56) + expand (:104-108, replace) */
static void or_pexpand(or_pnode *nd, const float *pol81) {
    int32_t leg[81];
    int nl = or_legal_actions(&nd->s, leg);
    float lp[81];
    for (int i = 0; i < nl; ++i) lp[i] = pol81[leg[i]];
    float sum = or_np_pairwise_sum_f32(lp, nl);
    int p64 = 0;
    if (sum > 0) {
        for (int i = 0; i < nl; ++i) lp[i] = lp[i] / sum;
    } else {
        p64 = 1;
    }
    for (int i = 0; i < nd->nch; ++i) or_pnode_free(nd->ch[i]);
    free(nd->ch);
    nd->ch = (or_pnode **)malloc(sizeof(or_pnode *) * (size_t)(nl ? nl : 1));
    nd->nch = nl;
    for (int i = 0; i < nl; ++i) {
        or_state ns;
        or_next(&nd->s, leg[i], &ns);
        or_pnode *c = or_pnode_new(&ns);
        c->p = p64 ? 0.0f : lp[i];
        c->p64 = p64;
        c->nsib = nl;
        nd->ch[i] = c;
    }
}

/* backpropagate (:111-116); is_f32: the value is the network's np.float32 */
static void or_pbackprop(or_pnode **path, int len, float value, int is_f32) {
    for (int i = len - 1; i >= 0; --i) {
        path[i]->w += value;
        if (is_f32) path[i]->w_f32 = 1;
        path[i]->n += 1;
        value = -value;
    }
}

/* next_child_node (:119-130) */
static or_pnode *or_pnext_child(or_pnode *nd) {
    int64_t t = 0;
    for (int i = 0; i < nd->nch; ++i) t += nd->ch[i]->n;
    const double sqt = sqrt((double)t);
    double best = 0.0;
    int bi = -1, best_nan = 0;
    for (int i = 0; i < nd->nch; ++i) {
        or_pnode *c = nd->ch[i];
        double v;
        if (c->p64) { /* np.float64 prior: the whole expression is float64 */
            const double p = 1.0 / (double)c->nsib;
            const double q = c->n ? (c->w_f32 ? (double)((-c->w) / (float)c->n) : (double)(-c->w) / (double)c->n) : 0.0;
            v = q + ((1.0 * p) * sqt) / (double)(1 + c->n);
        } else {        /* np.float32 prior: float32 ops, Python scalars cast to float32 */
            const float q = c->n ? (c->w_f32 ? (-c->w) / (float)c->n : (float)((double)(-c->w) / (double)c->n)) : 0.0f;
            const float u = ((1.0f * c->p) * (float)sqt) / (float)(1 + c->n);
            v = (double)(q + u);
        }
        if (best_nan) continue;
        if (v != v) { bi = i; best_nan = 1; continue; }
        if (bi < 0 || v > best) { best = v; bi = i; }
    }
    return bi < 0 ? NULL : nd->ch[bi];
}

/* search_leaf (:88-101): terminal -> returns -(-1 if lose else 0), a Python int */
static or_pnode *or_psearch_leaf(or_pnode *nd, or_pnode **path, int *len, float *value) {
    for (;;) {
        path[(*len)++] = nd;
        if (or_is_done(&nd->s)) {
            *value = or_is_lose(&nd->s) ? 1.0f : 0.0f;
            return nd;
        }
        if (nd->nch <= 0) { *value = 0.0f; return nd; }
        nd = or_pnext_child(nd);
    }
}

/* pv_mcts_scores (:133-181) with PV_EVALUATE_COUNT / MCTS_BATCH_SIZE as parameters.
 * Returns |root children|; scores_out = boltzman (Python floats) or one-hot. */
int or_pv_mcts_scores_py(const or_state *root_s, double temperature, int evaluate_count, int batch_size,
                         or_eval_fn eval, void *ctx, double *scores_out, int32_t *visits_out,
                         or_search_stats *st_out) {
    or_search_stats st;
    memset(&st, 0, sizeof(st));
    or_pnode *root = or_pnode_new(root_s);
    st.nodes = 1;
    int qcap = 64, qn = 0;
    or_pnode **qleaf = (or_pnode **)malloc(sizeof(or_pnode *) * (size_t)qcap);
    or_pnode ***qpath = (or_pnode ***)malloc(sizeof(or_pnode **) * (size_t)qcap);
    int *qlen = (int *)malloc(sizeof(int) * (size_t)qcap);
    or_pnode *path[OR_MAX_PATH];
    for (int i = 0; i < evaluate_count; ++i) {
        int len = 0;
        float value;
        or_pnode *leaf = or_psearch_leaf(root, path, &len, &value);
        if (len - 1 > st.max_depth) st.max_depth = len - 1;
        if (or_is_done(&leaf->s)) {
            or_pbackprop(path, len, value, 0);
            st.terminal++;
            continue;
        }
        if (leaf->n == 0) {
            if (qn == qcap) {
                qcap *= 2;
                qleaf = (or_pnode **)realloc(qleaf, sizeof(or_pnode *) * (size_t)qcap);
                qpath = (or_pnode ***)realloc(qpath, sizeof(or_pnode **) * (size_t)qcap);
                qlen = (int *)realloc(qlen, sizeof(int) * (size_t)qcap);
            }
            qleaf[qn] = leaf;
            qpath[qn] = (or_pnode **)malloc(sizeof(or_pnode *) * (size_t)len);
            memcpy(qpath[qn], path, sizeof(or_pnode *) * (size_t)len);
            qlen[qn] = len;
            qn++;
        }
        if (qn >= batch_size || i == evaluate_count - 1) {
            if (qn > 0) {
                st.flushes++;
                float *pols = (float *)malloc(sizeof(float) * 81 * (size_t)qn);
                float *vals = (float *)malloc(sizeof(float) * (size_t)qn);
                for (int j = 0; j < qn; ++j) { /* one model call for the batch */
                    float x[243];
                    or_tensor_nchw(&qleaf[j]->s, x);
                    eval(x, pols + 81 * j, vals + j, ctx);
                    st.evals++;
                }
                for (int j = 0; j < qn; ++j) {
                    or_pexpand(qleaf[j], pols + 81 * j);
                    or_pbackprop(qpath[j], qlen[j], vals[j], 1);
                    free(qpath[j]);
                }
                free(pols);
                free(vals);
                qn = 0;
            }
        }
    }
    int nout = root->nch > 0 ? root->nch : 0;
    for (int i = 0; i < nout; ++i)
        if (visits_out) visits_out[i] = root->ch[i]->n;
    if (temperature == 0.0) { /* np.argmax, one-hot float64 */
        int mi = 0;
        for (int i = 1; i < nout; ++i)
            if (root->ch[i]->n > root->ch[mi]->n) mi = i;
        for (int i = 0; i < nout; ++i) scores_out[i] = 0.0;
        if (nout) scores_out[mi] = 1.0;
    } else {              /* boltzman: [x ** (1 / T)] then x / sum(xs), Python floats */
        const double e = 1.0 / temperature;
        double sum = 0.0;
        for (int i = 0; i < nout; ++i) {
            scores_out[i] = pow((double)root->ch[i]->n, e);
        }
        for (int i = 0; i < nout; ++i) sum += scores_out[i];
        for (int i = 0; i < nout; ++i) scores_out[i] = scores_out[i] / sum;
    }
    for (int j = 0; j < qn; ++j) free(qpath[j]);
    free(qleaf);
    free(qpath);
    free(qlen);
    or_pnode_free(root);
    if (st_out) *st_out = st;
    return nout;
}

/* evaluate_network.py:33-51 play() for one game: players[0] moves when
 * is_first_player(), each move pv_mcts_action (pv_mcts.py:184-188) drawing
 * np.random.choice from RandomState(seed). Returns the first player's point
 * (first_player_point, :26-30) * 2 (0, 1 or 2); actions_out gets the moves. */
int or_evaluate_play(uint32_t seed, double temperature, int evaluate_count, int batch_size, or_eval_fn eval0,
                     void *ctx0, or_eval_fn eval1, void *ctx1, int32_t *actions_out, int32_t *n_actions) {
    or_mt mt;
    or_mt_seed(&mt, seed);
    or_state s;
    or_state_initial(&s);
    int na = 0;
    while (!or_is_done(&s)) {
        const int first = or_is_first_player(&s);
        double sc[81];
        int32_t leg[81];
        int nl = or_legal_actions(&s, leg);
        int n = or_pv_mcts_scores_py(&s, temperature, evaluate_count, batch_size, first ? eval0 : eval1,
                                     first ? ctx0 : ctx1, sc, NULL, NULL);
        if (n != nl) return -1;
        int idx = or_np_choice(&mt, sc, n);
        actions_out[na++] = leg[idx];
        or_state ns;
        or_next(&s, leg[idx], &ns);
        s = ns;
    }
    *n_actions = na;
    if (or_is_lose(&s)) return or_is_first_player(&s) ? 0 : 2;
    return 1;
}

/* the hash evaluator with a salt (a second, different deterministic player) */
void or_hash_eval_salted(const float *x, float *policy, float *value, uint64_t salt);
void or_eval_hash_salted_cb(const float *x, float *policy, float *value, void *ctx) {
    or_hash_eval_salted(x, policy, value, ctx ? *(const uint64_t *)ctx : 0ULL);
}

int or_pv_mcts_scores_py_hash(const or_state *root, double temperature, int evaluate_count, int batch_size,
                              uint64_t salt, double *scores_out, int32_t *visits_out, or_search_stats *st) {
    return or_pv_mcts_scores_py(root, temperature, evaluate_count, batch_size, or_eval_hash_salted_cb, &salt,
                                scores_out, visits_out, st);
}

int or_evaluate_play_hash(uint32_t seed, double temperature, int evaluate_count, int batch_size, uint64_t salt0,
                          uint64_t salt1, int32_t *actions_out, int32_t *n_actions) {
    return or_evaluate_play(seed, temperature, evaluate_count, batch_size, or_eval_hash_salted_cb, &salt0,
                            or_eval_hash_salted_cb, &salt1, actions_out, n_actions);
}

/* self_play.py:66-99 play(model) for one game, RandomState(seed): per ply the HWC
 * input, policies (float64, 0 for illegal actions) and value (first_player_value
 * at ply 0, then alternating, :20-25 / :94-97). Returns plies. */
int or_self_play_game_py(uint32_t seed, double temperature, int evaluate_count, int batch_size, or_eval_fn eval,
                         void *ctx, float *tensors_hwc, double *policies, int8_t *values, int max_plies) {
    or_mt mt;
    or_mt_seed(&mt, seed);
    or_state s;
    or_state_initial(&s);
    int np_ = 0;
    while (!or_is_done(&s)) {
        if (np_ >= max_plies) return -1;
        double sc[81];
        int32_t leg[81];
        int nl = or_legal_actions(&s, leg);
        int n = or_pv_mcts_scores_py(&s, temperature, evaluate_count, batch_size, eval, ctx, sc, NULL, NULL);
        if (n != nl) return -2;
        double *pol = policies + 81 * (size_t)np_;
        for (int a = 0; a < 81; ++a) pol[a] = 0.0;
        for (int i = 0; i < nl; ++i) pol[leg[i]] = sc[i];
        or_tensor_hwc(&s, tensors_hwc + 243 * (size_t)np_);
        int idx = or_np_choice(&mt, sc, n);
        or_state ns;
        or_next(&s, leg[idx], &ns);
        s = ns;
        ++np_;
    }
    int v = or_is_lose(&s) ? (or_is_first_player(&s) ? -1 : 1) : 0;
    for (int i = 0; i < np_; ++i) {
        values[i] = (int8_t)v;
        v = -v;
    }
    return np_;
}

int or_self_play_game_py_hash(uint32_t seed, double temperature, int evaluate_count, int batch_size, uint64_t salt,
                              float *tensors_hwc, double *policies, int8_t *values, int max_plies) {
    return or_self_play_game_py(seed, temperature, evaluate_count, batch_size, or_eval_hash_salted_cb, &salt,
                                tensors_hwc, policies, values, max_plies);
}

int or_state_size(void) { return (int)sizeof(or_state); }
int or_search_stats_size(void) { return (int)sizeof(or_search_stats); }
