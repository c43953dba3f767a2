// g2048_astar.hip -- the A* replay pre-fill search (src/state_space_search.py:46-131), host code.
//
// The reference's A_star is a best-first search over boards: a node's priority is
// FofN = -merge_score // 2 (:38-40), the open list is a PriorityQueue of (FofN, insertion
// counter, node) (:56,94) so ties pop in insertion order, a popped node whose board is in the
// closed list is skipped when the stored node's FofN is GREATER than its own (:78-81, the
// comparison as written), every popped node's children are the boards of its changing moves in
// up/down/left/right order, each with one spawn (Board2048.available_moves, board.py:138-145),
// and the search stops at the first popped board that holds the goal tile (:71-76).  Branchy,
// pointer-chasing work with one priority queue: a poor fit for the GPU,
// so it runs on the host and hands transitions to the device ring (g2048.astar).
//
// Spawns: Philox4x32-10 keyed (seed, game, expansion counter) -- the reference's numpy/random
// stream cannot be reproduced -- or, for parity with reference runs, "a 2 in the first empty
// cell" (the rule tests/golden/gen_astar_goldens.py patches into the reference).
#include <stdint.h>
#include <string.h>

#include <queue>
#include <unordered_map>
#include <vector>

#include "../../include/g2048.h"
#include "g2048_common.hpp"

namespace {

struct Node {
    uint8_t b[16];
    int64_t parent;
    int64_t score;  // Board2048._mergescore
    int8_t move;    // 0 up, 1 down, 2 left, 3 right (-1 at the root)
};

// Python's -score // 2 (floor division)
inline int64_t fofn(int64_t score) {
    const int64_t n = -score;
    return n >= 0 ? n / 2 : -((-n + 1) / 2);
}

// Slide one line of exponents toward index 0: equal neighbours merge once, front first
// (board.py:92-126 on values; tile 2^e + 2^e -> 2^(e+1), score += 2^(e+1)).
inline int64_t slide4(uint8_t* v) {
    uint8_t out[4] = {0, 0, 0, 0};
    int k = 0, prev = -1;
    int64_t gain = 0;
    for (int i = 0; i < 4; ++i) {
        if (!v[i]) continue;
        if (prev == v[i]) {
            out[k++] = (uint8_t)(v[i] + 1);
            gain += (int64_t)1 << (v[i] + 1);
            prev = -1;
        } else {
            if (prev >= 0) out[k++] = (uint8_t)prev;
            prev = v[i];
        }
    }
    if (prev >= 0) out[k++] = (uint8_t)prev;
    memcpy(v, out, 4);
    return gain;
}

// board.py:147-183: up = columns toward row 0, down = reversed columns, left = rows toward
// column 0, right = reversed rows.  Returns whether the board changed; gain = merge score.
bool move_board(const uint8_t* in, int act, uint8_t* out, int64_t& gain) {
    memcpy(out, in, 16);
    gain = 0;
    for (int line = 0; line < 4; ++line) {
        int idx[4];
        for (int k = 0; k < 4; ++k) {
            const int kk = (act == 1 || act == 3) ? 3 - k : k;
            idx[k] = act <= 1 ? kk * 4 + line : line * 4 + kk;
        }
        uint8_t v[4] = {in[idx[0]], in[idx[1]], in[idx[2]], in[idx[3]]};
        gain += slide4(v);
        for (int k = 0; k < 4; ++k) out[idx[k]] = v[k];
    }
    return memcmp(in, out, 16) != 0;
}

uint32_t philox10_host(uint32_t c[4], uint32_t k0, uint32_t k1, int w) {
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)c[0] * 0xD2511F53u, p1 = (uint64_t)c[2] * 0xCD9E8D57u;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
        c[0] = n0;
        c[1] = n1;
        c[2] = n2;
        c[3] = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c[w];
}

constexpr uint32_t DOMAIN_ASTAR = 1u;  // (the env's step / reset / sample use 0 / 2 / 3)

// One spawn on a board that just changed (board.py:41-51): the k-th empty cell row-major gets
// a 2 (exponent 1) or, with p = 0.5, a 4.
void spawn(uint8_t* b, int mode, uint64_t seed, uint64_t game, uint64_t counter) {
    int empties[16], n = 0;
    for (int i = 0; i < 16; ++i)
        if (!b[i]) empties[n++] = i;
    if (!n) return;
    if (mode == G2048_ASTAR_SPAWN_FIRST_EMPTY) {
        b[empties[0]] = 1;
        return;
    }
    uint32_t c[4] = {(uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)game,
                     (uint32_t)(game >> 32) | (DOMAIN_ASTAR << 30)};
    uint32_t cc[4];
    memcpy(cc, c, sizeof(c));
    const uint32_t uz = philox10_host(cc, (uint32_t)seed, (uint32_t)(seed >> 32), 2);
    const uint32_t uw = cc[3];
    const uint32_t k = (uint32_t)(((uint64_t)uz * (uint32_t)n) >> 32);
    b[empties[k]] = uw < 0x80000000u ? 2 : 1;
}

struct BoardKey {
    uint64_t lo, hi;
    bool operator==(const BoardKey& o) const { return lo == o.lo && hi == o.hi; }
};
struct BoardHash {
    size_t operator()(const BoardKey& k) const {
        return (size_t)(k.lo * 0x9E3779B97F4A7C15ull ^ (k.hi + 0x632BE59BD9B4E019ull));
    }
};
inline BoardKey key_of(const uint8_t* b) {
    BoardKey k;
    memcpy(&k.lo, b, 8);
    memcpy(&k.hi, b + 8, 8);
    return k;
}

struct QE {
    int64_t pri, counter, node;
    bool operator>(const QE& o) const {
        return pri != o.pri ? pri > o.pri : counter > o.counter;
    }
};

}  // namespace

extern "C" G2048_API int g2048_astar_search(const uint8_t* start, int64_t start_score,
                                            int goal_exp, uint64_t seed, uint64_t game,
                                            int spawn_mode, int64_t max_expansions,
                                            int64_t max_path, uint8_t* path_boards,
                                            uint8_t* path_moves, int64_t* path_scores,
                                            int64_t* path_len, int64_t* visited,
                                            int64_t* expanded, int* success) {
    if (!start || !path_boards || !path_moves || !path_scores || !path_len || !visited ||
        !expanded || !success || max_path < 0 || goal_exp <= 0 || goal_exp > 30)
        return g2048_fail(G2048_EINVAL, "astar_search: NULL argument or bad goal / max_path");
    if (spawn_mode != G2048_ASTAR_SPAWN_PHILOX && spawn_mode != G2048_ASTAR_SPAWN_FIRST_EMPTY)
        return g2048_fail(G2048_EINVAL, "astar_search: spawn_mode %d", spawn_mode);
    for (int i = 0; i < 16; ++i)
        if (start[i] > 30) return g2048_fail(G2048_EINVAL, "astar_search: exponent > 30");
    std::vector<Node> nodes;
    nodes.reserve(1024);
    Node root;
    memcpy(root.b, start, 16);
    root.parent = -1;
    root.score = start_score;
    root.move = -1;
    nodes.push_back(root);
    std::priority_queue<QE, std::vector<QE>, std::greater<QE>> open;
    open.push(QE{0, 0, 0});  // openlist.put((0, 0, current_node)) (:56)
    std::unordered_map<BoardKey, int64_t, BoardHash> closed;
    int64_t nvis = 1, nexp = 0, cur = 0;
    int ok = 0;
    bool capped = false;
    while (!open.empty()) {
        cur = open.top().node;
        open.pop();
        ++nvis;
        const Node& c = nodes[(size_t)cur];
        bool goal = false;
        for (int i = 0; i < 16; ++i) goal = goal || c.b[i] == goal_exp;
        if (goal) {
            ok = 1;
            break;
        }
        const BoardKey key = key_of(c.b);
        auto it = closed.find(key);
        if (it != closed.end() && fofn(nodes[(size_t)it->second].score) > fofn(c.score)) continue;
        closed[key] = cur;
        if (max_expansions > 0 && nexp >= max_expansions) {
            capped = true;
            break;
        }
        uint8_t child[16];
        for (int act = 0; act < 4; ++act) {
            int64_t gain;
            const Node& p = nodes[(size_t)cur];  // (re-read: push_back may reallocate)
            if (!move_board(p.b, act, child, gain)) continue;
            ++nexp;
            spawn(child, spawn_mode, seed, game, (uint64_t)nexp);
            Node n;
            memcpy(n.b, child, 16);
            n.parent = cur;
            n.score = p.score + gain;
            n.move = (int8_t)act;
            nodes.push_back(n);
            open.push(QE{fofn(n.score), nexp, (int64_t)nodes.size() - 1});
        }
    }
    (void)capped;
    // the returned node is the last popped one (success or not), as in the reference (:71-101)
    int64_t len = 0;
    for (int64_t n = cur; nodes[(size_t)n].parent >= 0; n = nodes[(size_t)n].parent) ++len;
    if (len > max_path)
        return g2048_fail(G2048_EINVAL, "astar_search: path of %lld moves > max_path %lld",
                          (long long)len, (long long)max_path);
    int64_t n = cur;
    for (int64_t k = len; k >= 0; --k) {
        memcpy(path_boards + 16 * k, nodes[(size_t)n].b, 16);
        path_scores[k] = nodes[(size_t)n].score;
        if (k > 0) path_moves[k - 1] = (uint8_t)nodes[(size_t)n].move;
        n = nodes[(size_t)n].parent;
    }
    *path_len = len;
    *visited = nvis;
    *expanded = nexp;
    *success = ok;
    return G2048_OK;
}
