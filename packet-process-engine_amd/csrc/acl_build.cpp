/*
 * acl_build.cpp — host-side compiler from the PPE rule list to the device classifier image (ppe_image.h).
 *
 * Replaces the absent DP_Acl_Load_Rule tree build (called at dataplane/src/common/dp_cmd.c:2019; sources
 * dp_acl.c/acl64.c missing, dataplane/src/acl/acl.mk:13-15).  Algorithm: HyperSplit-style recursive
 * partitioning of the 5-D header space (sip, dip, sport, dport, proto), one binary split per node at a rule
 * boundary, chosen to minimise the larger child's rule count.  Exactness invariant (lowest-index first match,
 * SURVEY.md §8(a) A11): every node keeps, in ascending rule index, every rule whose box intersects its region,
 * truncated after the first rule whose box covers the region and has no residual (MAC / time) constraint — no
 * later rule can ever win inside that region.  A leaf therefore holds exactly the candidates that can match
 * there, in priority order, and the kernel returns the first one that matches.
 *
 * Rule semantics (frozen here; the reference engine is absent):
 *   entry eligible iff used == NULL || used[i] == RULE_ENTRY_STATUS_USED
 *   sip matches iff sip_mask == 0 || top sip_mask bits of (pkt.sip ^ rule.sip) are zero   (prefix length 0..32)
 *   dip likewise; sport/dport/protocol: start <= x <= end (an empty range never matches)
 *   smac/dmac: all-zero = any, else equal; time: (0,0) = any, else time_start <= ts <= time_end
 *   action: the rule's action word; the packet is dropped iff it equals ACL_RULE_ACTION_DROP (flow.c:232)
 */
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <deque>
#include <vector>

#include "ppe_hip.h"
#include "ppe_image.h"
#include "ppe_internal.h"

namespace {

struct Rule {
    uint32_t lo[PPE_NDIMS], hi[PPE_NDIMS];
    uint32_t id;
    uint32_t action;
    uint32_t resid;
    uint32_t slot;
};

struct Work {
    uint32_t node;
    uint32_t depth;
    uint32_t lo[PPE_NDIMS], hi[PPE_NDIMS];
    std::vector<uint32_t> rules;  // slots, ascending
};

inline bool covers(const Rule &r, const uint32_t *lo, const uint32_t *hi) {
    for (int d = 0; d < PPE_NDIMS; ++d)
        if (r.lo[d] > lo[d] || r.hi[d] < hi[d]) return false;
    return true;
}

inline uint32_t prefix_lo(uint32_t ip, uint32_t len) {
    return len == 0 ? 0u : (ip & (0xffffffffu << (32 - len)));
}
inline uint32_t prefix_hi(uint32_t ip, uint32_t len) {
    return len == 0 ? 0xffffffffu : (prefix_lo(ip, len) | ~(0xffffffffu << (32 - len)));
}

inline bool mac_nonzero(const uint8_t *m) {
    return (m[0] | m[1] | m[2] | m[3] | m[4] | m[5]) != 0;
}
inline uint32_t mac_lo(const uint8_t *m) {
    return (uint32_t)m[0] | ((uint32_t)m[1] << 8) | ((uint32_t)m[2] << 16) | ((uint32_t)m[3] << 24);
}
inline uint32_t mac_hi(const uint8_t *m) { return (uint32_t)m[4] | ((uint32_t)m[5] << 8); }

struct TNode {
    uint32_t thr;    // internal: split threshold
    uint32_t left;   // internal: left child index (right = left + 1)
    uint32_t dim;    // split dimension, PPE_NODE_LEAF for a leaf
    uint32_t first;  // leaf: first entry in `leaf`
    uint32_t cnt;    // leaf: number of candidates
};

struct Forest {
    std::vector<TNode> nodes;  // BFS over every root: roots first, children contiguous and after their parent
    std::vector<uint32_t> leaf;
    uint32_t max_depth = 0, n_leaves = 0, max_leaf = 0, n_roots = 0;
    double depth_sum = 0;
    std::vector<uint32_t> runs;  // jump root: buckets per root, in bucket order
    double avg_depth() const { return n_leaves ? depth_sum / n_leaves : 0.0; }
};

// Jump (cut) root: bucket b = key[dim] >> shift, 2^bits buckets, each the root of its own subtree
struct Jump {
    uint32_t dim = 0, shift = 0, bits = 0;
};

Work full_box(const std::vector<Rule> &R) {
    Work w;
    w.node = 0;
    w.depth = 0;
    w.lo[0] = w.lo[1] = w.lo[2] = w.lo[3] = w.lo[4] = 0;
    w.hi[0] = w.hi[1] = 0xffffffffu;
    w.hi[2] = w.hi[3] = 0xffffu;
    w.hi[4] = 0xffu;
    w.rules.resize(R.size());
    for (uint32_t s = 0; s < R.size(); ++s) w.rules[s] = s;
    return w;
}

// The cut's buckets as subtree roots: every bucket gets the rules whose box meets it (ascending, closed after the
// first unconditional cover); a run of consecutive buckets with the same rule list shares one subtree, built over
// the run's union box (a classifier correct for the union is correct for each bucket in it).
// Returns one Work per run, and each run's bucket count in `runs`.
std::vector<Work> cut_roots(const std::vector<Rule> &R, const Jump &j, std::vector<uint32_t> &runs) {
    const uint32_t nb = 1u << j.bits;
    std::vector<std::vector<uint32_t>> lists(nb);
    std::vector<uint8_t> closed(nb, 0);
    Work box = full_box({});
    for (uint32_t s = 0; s < R.size(); ++s) {
        const Rule &r = R[s];
        const uint32_t b0 = r.lo[j.dim] >> j.shift, b1 = r.hi[j.dim] >> j.shift;
        for (uint32_t b = b0; b <= b1; ++b) {
            if (closed[b]) continue;
            lists[b].push_back(s);
            box.lo[j.dim] = b << j.shift;
            box.hi[j.dim] = box.lo[j.dim] | ((1u << j.shift) - 1u);
            if (r.resid == 0 && covers(r, box.lo, box.hi)) closed[b] = 1;
        }
    }
    std::vector<Work> roots;
    for (uint32_t b = 0; b < nb;) {
        uint32_t e = b + 1;
        while (e < nb && lists[e] == lists[b]) ++e;
        Work w = full_box({});
        w.lo[j.dim] = b << j.shift;
        w.hi[j.dim] = ((e - 1u) << j.shift) | ((1u << j.shift) - 1u);
        w.rules = std::move(lists[b]);
        runs.push_back(e - b);
        roots.push_back(std::move(w));
        b = e;
    }
    return roots;
}

// HyperSplit partitioning of every root box, breadth-first over the whole forest (so the nodes of depth < L are a
// prefix of the node array for every L: the LDS-staged top of the image is whole levels)
Forest build_forest(const std::vector<Rule> &R, std::vector<Work> roots, uint32_t binth) {
    Forest f;
    // analysis knob (tools/walk_depth.py, not a product setting): a node at depth >= PPE_LEAF_CAP_DEPTH with at most
    // PPE_LEAF_CAP_N candidates becomes a leaf list, bounding the depth of the walk's tail
    static const uint32_t cap_depth = (uint32_t)std::max(0, std::atoi(std::getenv("PPE_LEAF_CAP_DEPTH") ? std::getenv("PPE_LEAF_CAP_DEPTH") : "0"));
    static const uint32_t cap_leaf = (uint32_t)std::max(1, std::atoi(std::getenv("PPE_LEAF_CAP_N") ? std::getenv("PPE_LEAF_CAP_N") : "1"));
    std::vector<TNode> &nodes = f.nodes;
    const size_t node_budget = PPE_NODE_MAX - 2;
    std::deque<Work> q;
    f.n_roots = (uint32_t)roots.size();
    nodes.resize(roots.size());
    for (uint32_t i = 0; i < roots.size(); ++i) {
        roots[i].node = i;
        roots[i].depth = 0;
        q.push_back(std::move(roots[i]));
    }
    std::vector<uint32_t> clo, chi, cand;
    while (!q.empty()) {
        Work w = std::move(q.front());
        q.pop_front();

        // redundancy removal: drop everything after the first unconditional cover of this region
        std::vector<uint32_t> S;
        S.reserve(w.rules.size());
        for (uint32_t s : w.rules) {
            S.push_back(s);
            if (R[s].resid == 0 && covers(R[s], w.lo, w.hi)) break;
        }
        w.rules.clear();
        w.rules.shrink_to_fit();

        auto make_leaf = [&](const std::vector<uint32_t> &L) {
            TNode &nd = nodes[w.node];
            nd.dim = PPE_NODE_LEAF;
            nd.first = (uint32_t)f.leaf.size();
            nd.cnt = (uint32_t)L.size();
            f.leaf.insert(f.leaf.end(), L.begin(), L.end());
            ++f.n_leaves;
            f.max_leaf = std::max(f.max_leaf, (uint32_t)L.size());
            f.depth_sum += w.depth;
            if (w.depth > f.max_depth) f.max_depth = w.depth;
        };

        const bool first_certain = !S.empty() && R[S[0]].resid == 0 && covers(R[S[0]], w.lo, w.hi);
        if (S.empty() || first_certain || S.size() <= binth || w.depth + 1 >= PPE_MAX_DEPTH ||
            (cap_depth && w.depth >= cap_depth && S.size() <= cap_leaf) ||
            nodes.size() + 2 > node_budget) {
            if (first_certain) S.resize(1);
            make_leaf(S);
            continue;
        }

        // choose (dim, threshold) minimising (max(|left|,|right|), |left|+|right|)
        int best_d = -1;
        uint32_t best_t = 0;
        size_t best_max = SIZE_MAX, best_sum = SIZE_MAX;
        for (int d = 0; d < PPE_NDIMS; ++d) {
            clo.clear();
            chi.clear();
            cand.clear();
            for (uint32_t s : S) {
                uint32_t l = std::max(R[s].lo[d], w.lo[d]);
                uint32_t h = std::min(R[s].hi[d], w.hi[d]);
                clo.push_back(l);
                chi.push_back(h);
                if (l > w.lo[d]) cand.push_back(l - 1);
                if (h < w.hi[d]) cand.push_back(h);
            }
            if (cand.empty()) continue;
            std::sort(clo.begin(), clo.end());
            std::sort(chi.begin(), chi.end());
            std::sort(cand.begin(), cand.end());
            cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
            for (uint32_t t : cand) {
                size_t left = (size_t)(std::upper_bound(clo.begin(), clo.end(), t) - clo.begin());
                size_t right = S.size() - (size_t)(std::upper_bound(chi.begin(), chi.end(), t) - chi.begin());
                size_t mx = std::max(left, right), sm = left + right;
                if (mx < best_max || (mx == best_max && sm < best_sum)) {
                    best_max = mx;
                    best_sum = sm;
                    best_d = d;
                    best_t = t;
                }
            }
        }
        if (best_d < 0) {  // cannot happen: S[0] does not cover the region, so it has a boundary inside it
            make_leaf(S);
            continue;
        }

        // a threshold is l - 1 (l > region lo) or h (h < region hi): never 0xffffffff, the leaf marker
        const uint32_t left_idx = (uint32_t)nodes.size();
        nodes.resize(nodes.size() + 2);
        nodes[w.node].thr = best_t;
        nodes[w.node].left = left_idx;
        nodes[w.node].dim = (uint32_t)best_d;

        Work L, Rt;
        L.node = left_idx;
        Rt.node = left_idx + 1;
        L.depth = Rt.depth = w.depth + 1;
        std::memcpy(L.lo, w.lo, sizeof w.lo);
        std::memcpy(L.hi, w.hi, sizeof w.hi);
        std::memcpy(Rt.lo, w.lo, sizeof w.lo);
        std::memcpy(Rt.hi, w.hi, sizeof w.hi);
        L.hi[best_d] = best_t;
        Rt.lo[best_d] = best_t + 1;
        for (uint32_t s : S) {
            if (R[s].lo[best_d] <= best_t) L.rules.push_back(s);
            if (R[s].hi[best_d] > best_t) Rt.rules.push_back(s);
        }
        q.push_back(std::move(L));
        q.push_back(std::move(Rt));
    }
    return f;
}

// ---- cut lists (image v7, ppe_image.h) ----
struct CutLists {
    uint32_t b0 = 0, b1 = 0, max_len = 0;
    std::vector<uint8_t> len;        // per bucket
    std::vector<uint32_t> entries;   // rule slots, bucket after bucket, each bucket's in priority order
    size_t n_entries = 0;
};

// The lists of the cut (b0 sip bits, b1 dip bits): per bucket, the rules whose box meets it in ascending index,
// closed after the first rule that covers the whole bucket for every key that reaches the ACL on the classify path
// (every sport / dport, protocols 6 and 17).  False when a list would exceed PPE_CUT_MAX_LIST entries or the work
// (buckets visited) the budget.  store = false: the list lengths only (the width search), no entries.
bool cut_lists(const std::vector<Rule> &R, uint32_t b0, uint32_t b1, size_t budget, CutLists &out, bool store) {
    const uint32_t nb = 1u << (b0 + b1);
    std::vector<uint8_t> len(nb, 0), closed(nb, 0);
    std::vector<std::vector<uint32_t>> lists(store ? nb : 0u);
    size_t n_ent = 0;
    size_t visits = 0;
    uint32_t max_len = 0;
    const uint64_t w0 = 1ull << (32 - b0), w1 = 1ull << (32 - b1);  // keys per bucket row / column
    for (uint32_t s = 0; s < R.size(); ++s) {
        const Rule &r = R[s];
        const uint32_t x0 = b0 ? r.lo[PPE_DIM_SIP] >> (32 - b0) : 0u, x1 = b0 ? r.hi[PPE_DIM_SIP] >> (32 - b0) : 0u;
        const uint32_t y0 = b1 ? r.lo[PPE_DIM_DIP] >> (32 - b1) : 0u, y1 = b1 ? r.hi[PPE_DIM_DIP] >> (32 - b1) : 0u;
        const bool ports_all = r.lo[PPE_DIM_SPORT] == 0u && r.hi[PPE_DIM_SPORT] == 0xffffu &&
                               r.lo[PPE_DIM_DPORT] == 0u && r.hi[PPE_DIM_DPORT] == 0xffffu &&
                               r.lo[PPE_DIM_PROTO] <= 6u && r.hi[PPE_DIM_PROTO] >= 17u;
        for (uint32_t x = x0; x <= x1; ++x) {
            // the rule covers bucket row x iff its sip range holds the row's whole key range
            const bool cx = (uint64_t)r.lo[PPE_DIM_SIP] <= x * w0 && (uint64_t)r.hi[PPE_DIM_SIP] >= x * w0 + w0 - 1u;
            for (uint32_t y = y0; y <= y1; ++y) {
                if (++visits > budget) return false;
                const uint32_t b = (x << b1) | y;
                if (closed[b]) continue;
                if (++len[b] > PPE_CUT_MAX_LIST) return false;
                if (store) lists[b].push_back(s);
                ++n_ent;
                max_len = std::max(max_len, (uint32_t)len[b]);
                const bool cy = (uint64_t)r.lo[PPE_DIM_DIP] <= y * w1 && (uint64_t)r.hi[PPE_DIM_DIP] >= y * w1 + w1 - 1u;
                if (ports_all && cx && cy) closed[b] = 1;
            }
        }
    }
    out.b0 = b0;
    out.b1 = b1;
    out.max_len = max_len;
    out.len = std::move(len);
    out.entries.clear();
    out.n_entries = n_ent;
    if (store)
        for (uint32_t b = 0; b < nb; ++b) out.entries.insert(out.entries.end(), lists[b].begin(), lists[b].end());
    return true;
}

// Pick the cut: every split of T = b0 + b1 <= PPE_CUT_MAX_BITS bits between sip and dip (each >= 2), by the expected
// entries a lookup reads (half for a uniformly random key: entries / buckets; half for a key inside a rule's box, the
// size-biased list length sum(len^2) / entries), plus a little for the longest list (the wave's trip count) and for
// every bit (LDS), a quarter of that when the whole cut fits half a CU's LDS (no L2 reads at all).
// PPE_CUT_BITS=T (tests, A/B) fixes the total.  False when no cut qualifies (a list longer than 15 entries at every
// width: then the classify kernel walks the tree).
bool choose_cut(const std::vector<Rule> &R, bool ids16, CutLists &best, bool &lds_fit) {
    const char *fb = std::getenv("PPE_CUT_BITS");
    const int force = fb && *fb ? std::atoi(fb) : -1;
    const size_t budget = 16u * (R.size() + 1u) + (1u << PPE_CUT_MAX_BITS);
    double cbest = 1e30;
    uint32_t bb0 = 0, bb1 = 0;
    bool found = false;
    lds_fit = false;
    for (uint32_t T = 5; T <= PPE_CUT_MAX_BITS; ++T) {
        if (force >= 0 && (int)T != force) continue;
        for (uint32_t b0 = 3; b0 + 2 <= T; ++b0) {  // (b0 >= 3, b1 >= 2: the flag bits below the relative prefixes)
            CutLists c;
            if (!cut_lists(R, b0, T - b0, budget, c, false)) continue;
            const double nb = (double)(1u << T), ne = (double)c.n_entries;
            double sq = 0;
            for (uint8_t l : c.len) sq += (double)l * l;
            // groups (20 B per 32 buckets), 4-bit fingerprints, 16-B entries and 2-B ids in half a CU's LDS (two
            // 1024-thread workgroups, the counter bins and the staging's 1-KB rounding beside them): the whole lookup
            // runs from LDS, no L2 round
            const bool lds = 0.625 * nb + 18.5 * ne + 3.0 * 1024 <= 80.0 * 1024 && ids16;
            const double cost = (0.5 * ne / nb + 0.5 * (ne ? sq / ne : 0.0) + 0.02 * c.max_len + 0.01 * T) *
                                (lds ? 0.25 : 1.0);
            if (std::getenv("PPE_ACL_DEBUG"))
                std::fprintf(stderr, "acl_build: cut sip %u dip %u: entries %zu max %u cost %.3f\n", b0, T - b0,
                             c.n_entries, c.max_len, cost);
            if (cost < cbest - 1e-9) {
                cbest = cost;
                bb0 = b0;
                bb1 = T - b0;
                found = true;
                lds_fit = lds;
            }
        }
    }
    return found && cut_lists(R, bb0, bb1, budget, best, true);
}

}  // namespace

extern "C" int ppe_acl_build_image(const RCP_BLOCK_ACL_RULE_TUPLE *rules, const uint8_t *used, uint32_t n,
                                   uint32_t default_action, uint32_t binth, uint32_t **words_out,
                                   uint32_t *n_words_out, ppe_acl_stats_t *st) {
    if (!words_out || !n_words_out) return PPE_EINVAL;
    if (n && !rules) return PPE_EINVAL;
    if (n > (1u << 24)) return PPE_EINVAL;
    if (binth == 0) binth = 1;  // one candidate per leaf: deepest tree, shortest scan (fastest measured)
    auto t0 = std::chrono::steady_clock::now();

    // ---- compile eligible rules to boxes (slot order = ascending rule index) ----
    std::vector<Rule> R;
    std::vector<uint32_t> resid_words;
    R.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
        if (used && used[i] != RULE_ENTRY_STATUS_USED) continue;
        const RCP_BLOCK_ACL_RULE_TUPLE &t = rules[i];
        if (t.sip_mask > 32 || t.dip_mask > 32) return PPE_EINVAL;  // parsers reject these (rule/rule.c:63-73)
        if (t.sport_start > t.sport_end || t.dport_start > t.dport_end || t.protocol_start > t.protocol_end)
            continue;  // empty range: can never match
        Rule r;
        r.lo[PPE_DIM_SIP] = prefix_lo(t.sip, t.sip_mask);
        r.hi[PPE_DIM_SIP] = prefix_hi(t.sip, t.sip_mask);
        r.lo[PPE_DIM_DIP] = prefix_lo(t.dip, t.dip_mask);
        r.hi[PPE_DIM_DIP] = prefix_hi(t.dip, t.dip_mask);
        r.lo[PPE_DIM_SPORT] = t.sport_start;
        r.hi[PPE_DIM_SPORT] = t.sport_end;
        r.lo[PPE_DIM_DPORT] = t.dport_start;
        r.hi[PPE_DIM_DPORT] = t.dport_end;
        r.lo[PPE_DIM_PROTO] = t.protocol_start;
        r.hi[PPE_DIM_PROTO] = t.protocol_end;
        r.id = i;
        r.action = t.action;
        r.resid = 0;
        if (mac_nonzero(t.dmac)) r.resid |= PPE_RESID_DMAC;
        if (mac_nonzero(t.smac)) r.resid |= PPE_RESID_SMAC;
        if (t.time_start != 0 || t.time_end != 0) r.resid |= PPE_RESID_TIME;
        r.slot = (uint32_t)R.size();
        R.push_back(r);
        uint32_t rw[8] = {mac_lo(t.dmac), mac_hi(t.dmac), mac_lo(t.smac), mac_hi(t.smac),
                          (uint32_t)t.time_start, (uint32_t)(t.time_start >> 32),
                          (uint32_t)t.time_end, (uint32_t)(t.time_end >> 32)};
        resid_words.insert(resid_words.end(), rw, rw + 8);
    }

    // ---- the root: a cut on the top bits of one dimension (jump table) or a single split tree ----
    const Forest base = build_forest(R, {full_box(R)}, binth);
    Forest best = base;
    Jump jbest;  // bits == 0: no jump table
    if (!base.nodes.empty() && base.nodes[0].dim != PPE_NODE_LEAF) {
        // cut the dimension the plain tree splits first; try a few widths, keep the cheapest: walk levels (the
        // fixed-trip LDS walk pays the deepest leaf, the per-lane global walk the average; the table read counts
        // as a level) plus one level per 16 KB of nodes and table (LDS footprint: fewer image copies per CU).
        // Measured on MI355X (C1 / C4, two-stream pipeline): 10 bits beat 0, 8 and 12.
        const uint32_t jd = base.nodes[0].dim;
        const uint32_t width = jd <= PPE_DIM_DIP ? 32u : (jd <= PPE_DIM_DPORT ? 16u : 8u);
        auto cost = [](const Forest &f, uint32_t bits) {
            const double bytes = 16.0 * f.nodes.size() + (bits ? 4.0 * (1u << bits) : 0.0);
            return 0.5 * (f.max_depth + 1) + 0.5 * (f.avg_depth() + 1) + (bits ? 1.0 : 0.0) + bytes / 16384.0;
        };
        double cbest = cost(base, 0);
        // PPE_JUMP_BITS (tuning / experiments): 0 = never cut, k = cut exactly k bits
        const char *fj = std::getenv("PPE_JUMP_BITS");
        const int force = fj && *fj ? std::atoi(fj) : -1;
        if (force >= 0) cbest = 1e30;
        for (uint32_t bits : {4u, 6u, 8u, 10u, 12u}) {
            if (bits >= width || force == 0) break;
            if (force > 0 && (int)bits != force) continue;
            if (force < 0 && bits > 8 && base.nodes.size() > 65536) break;  // large sets: wide cuts only replicate
            Jump j = {jd, width - bits, bits};
            std::vector<uint32_t> runs;
            std::vector<Work> roots = cut_roots(R, j, runs);
            Forest f = build_forest(R, std::move(roots), binth);
            f.runs = std::move(runs);
            if (force < 0 && f.nodes.size() > 2 * base.nodes.size() + (1u << bits) + 64u) continue;  // blow-up
            const double c = cost(f, bits);
            if (std::getenv("PPE_ACL_DEBUG"))
                std::fprintf(stderr, "acl_build: jump dim %u bits %u: nodes %zu max_depth %u avg %.2f cost %.2f\n",
                             jd, bits, f.nodes.size(), f.max_depth, f.avg_depth(), c);
            if (c < cbest - 1e-9) {
                cbest = c;
                best = std::move(f);
                jbest = j;
            }
        }
    }
    if (best.nodes.size() > PPE_NODE_MAX - 2) return PPE_ENOMEM;
    std::vector<TNode> &nodes = best.nodes;
    std::vector<uint32_t> &leaf = best.leaf;
    const uint32_t max_depth = best.max_depth, n_leaves = best.n_leaves, max_leaf = best.max_leaf;
    const double depth_sum = best.depth_sum;

    // ---- assemble the image ----
    const uint32_t n_nodes = (uint32_t)nodes.size();
    const uint32_t n_slots = (uint32_t)R.size();  // + the sentinel at slot n_slots
    // leaf list section: only when some leaf holds more than one candidate (else the payload is the rule slot)
    std::vector<uint32_t> lwords;
    if (max_leaf > 1) {
        for (TNode &nd : nodes) {
            if (nd.dim != PPE_NODE_LEAF) continue;
            const uint32_t first = (uint32_t)lwords.size();
            if (nd.cnt >= PPE_LEAF_CNT_ESC) lwords.push_back(nd.cnt);  // long list: its length leads the entries
            lwords.insert(lwords.end(), leaf.begin() + nd.first, leaf.begin() + nd.first + nd.cnt);
            nd.first = first;
        }
    }
    const uint32_t n_jump = jbest.bits ? 1u << jbest.bits : 0u;
    const uint32_t off_nodes = PPE_IMG_HDR_WORDS + n_jump;  // the jump table (if any) sits between header and nodes
    const uint32_t off_leaf = off_nodes + PPE_NODE_WORDS * n_nodes;
    uint32_t off_rules = off_leaf + (uint32_t)lwords.size();
    off_rules = (off_rules + 7u) & ~7u;
    // residual (MAC / time) records only when some rule has one: the kernel reads them only for such rules
    bool any_resid = false;
    for (const Rule &r : R) any_resid |= r.resid != 0;
    const uint32_t off_resid = off_rules + 8u * (n_slots + 1u);
    const uint32_t end_resid = off_resid + (any_resid ? 8u * (n_slots + 1u) : 0u);

    // ---- 2-level blocks (block section, ppe_image.h): breadth-first over the forest's roots ----
    auto is_leaf = [&](uint32_t x) { return nodes[x].dim == PPE_NODE_LEAF; };
    auto c0 = [&](uint32_t x) { return is_leaf(x) ? x : nodes[x].left; };
    auto c1 = [&](uint32_t x) { return is_leaf(x) ? x : nodes[x].left + 1u; };
    auto thr = [&](uint32_t x) { return is_leaf(x) ? 0xffffffffu : nodes[x].thr; };  // leaf: pass-through
    auto kslot = [&](uint32_t x) { return is_leaf(x) ? 0u : nodes[x].dim; };
    // compact leaves (v6, ppe_image.h): one candidate per leaf and no residual fields; PPE_COMPACT=0 turns them off
    // (A/B and tests of the v5 leaf path)
    const char *ce = std::getenv("PPE_COMPACT");
    const bool compact = max_leaf <= 1 && !any_resid && !(ce && *ce == '0');
    auto cx_flags = [&](uint32_t slot) -> uint32_t {  // the compact exit's flag bits for the candidate in `slot`
        if (slot == n_slots)  // the sentinel
            return PPE_CX_NOHIT | PPE_CX_TCP | PPE_CX_UDP | (default_action == ACL_RULE_ACTION_DROP ? PPE_CX_DROP : 0u);
        const Rule &r = R[slot];
        uint32_t f = r.action == ACL_RULE_ACTION_DROP ? PPE_CX_DROP : 0u;
        if (r.lo[PPE_DIM_PROTO] <= 6u && 6u <= r.hi[PPE_DIM_PROTO]) f |= PPE_CX_TCP;
        if (r.lo[PPE_DIM_PROTO] <= 17u && 17u <= r.hi[PPE_DIM_PROTO]) f |= PPE_CX_UDP;
        if (r.lo[PPE_DIM_SIP] == r.hi[PPE_DIM_SIP]) f |= PPE_CX_S32;
        if (r.lo[PPE_DIM_DIP] == r.hi[PPE_DIM_DIP]) f |= PPE_CX_D32;
        return f;
    };
    auto leaf_exit = [&](uint32_t x) -> uint32_t {
        const TNode &nd = nodes[x];
        if (max_leaf > 1) return PPE_BLK_LEAF | nd.first | (std::min(nd.cnt, PPE_LEAF_CNT_ESC) << 23);
        const uint32_t slot = nd.cnt ? leaf[nd.first] : n_slots;
        return PPE_BLK_LEAF | slot | (compact ? cx_flags(slot) : 0u);
    };
    if (max_leaf > 1 && lwords.size() >= (1u << 23)) return PPE_ENOMEM;  // leaf exits hold 23-bit list offsets
    // 2-level blocks (ppe_image.h block section): position p of a block holds node pos[p] (p's children are 2p + 1
    // and 2p + 2); a leaf passes through (threshold ~0, both children itself); the 4 exits lead to the next blocks
    // or carry leaf payloads.  Breadth-first from every root.
    std::vector<uint32_t> bwords;
    uint32_t max_bdepth = 1;
    auto build_blocks = [&]() {
        constexpr uint32_t npos = 3u, bw = PPE_BLK_WORDS;
        std::vector<uint32_t> bnode, bdepth;
        bwords.clear();
        max_bdepth = 1;
        auto add_block = [&](uint32_t x, uint32_t d) {
            bnode.push_back(x);
            bdepth.push_back(d);
            bwords.resize(bwords.size() + bw, 0u);
            return (uint32_t)bnode.size() - 1u;
        };
        for (uint32_t r = 0; r < best.n_roots; ++r) add_block(r, 1u);
        uint32_t pos[npos];
        for (size_t bi = 0; bi < bnode.size(); ++bi) {  // blocks appended while scanning: breadth-first order
            pos[0] = bnode[bi];
            for (uint32_t q = 1; q < npos; ++q) pos[q] = (q & 1u) ? c0(pos[(q - 1u) / 2u]) : c1(pos[(q - 1u) / 2u]);
            uint32_t slots = 0;
            for (uint32_t q = 0; q < npos; ++q) {
                bwords[bi * bw + q] = thr(pos[q]);
                slots |= kslot(pos[q]) << (4u * q);
            }
            bwords[bi * bw + npos] = slots;
            for (uint32_t e = 0; e <= npos; ++e) {  // (add_block may reallocate bwords: index, not a pointer)
                const uint32_t par = pos[npos / 2u + (e >> 1)];
                const uint32_t ch = (e & 1u) ? c1(par) : c0(par);
                uint32_t v;
                if (is_leaf(ch)) {
                    v = leaf_exit(ch);
                } else {
                    v = add_block(ch, bdepth[bi] + 1u);
                    max_bdepth = std::max(max_bdepth, bdepth[bi] + 1u);
                }
                bwords[bi * bw + npos + 1u + e] = v;
            }
        }
        return (uint32_t)bnode.size();
    };
    // (3-level 64-B blocks, an option until round 4, take one L2 round trip per three levels instead of two but
    // measured slower on C3: the 64-B block in flight per lane and tile costs the registers of more tiles)
    const uint32_t n_blocks = build_blocks();
    if (n_blocks >= PPE_BLK_LEAF) return PPE_ENOMEM;
    const uint32_t off_bsec = (end_resid + 7u) & ~7u;
    const uint32_t off_blocks = (off_bsec + n_jump + 7u) & ~7u;  // 32-B aligned blocks
    // compact records and the slot → index table follow the blocks, so the block section and the records they lead
    // to are one contiguous range (the multi-tile kernel stages it whole when it fits the CU's LDS)
    bool holes = false;
    for (uint32_t sl = 0; sl < n_slots; ++sl) holes |= R[sl].id != sl;
    const uint32_t off_crec = compact ? off_blocks + (uint32_t)bwords.size() : 0u;
    const uint32_t off_idtab = compact && holes ? off_crec + PPE_CREC_WORDS * (n_slots + 1u) : 0u;
    // (the index table has an entry for the sentinel slot too: crec_check reads idtab[slot] for every leaf)
    const uint32_t end_tree = !compact ? off_blocks + (uint32_t)bwords.size()
                              : off_idtab ? off_idtab + ((n_slots + 1u + 3u) & ~3u)
                                          : off_crec + PPE_CREC_WORDS * (n_slots + 1u);
    // ---- the cut-list section (v7): a classifier of its own for the classify kernel, after the tree ----
    CutLists cut;
    const char *cenv = std::getenv("PPE_CUT");
    const bool want_cut = !any_resid && !(cenv && *cenv == '0');
    // rule ids in 16-bit words when every index fits (R is in index order: its last id is the largest)
    const bool ids16 = R.empty() || R.back().id < 0x10000u;
    bool lds_fit = false;
    const bool have_cut = want_cut && choose_cut(R, ids16, cut, lds_fit) && cut.entries.size() < (1u << 25);  // (< 1 GB)
    // entry lines with in-line ids for cuts read from L2 (the id read after a match hits L1); dense entries and a
    // separate id array for those that fit LDS (where the id read costs nothing and lines would waste room)
    const char *lenv = std::getenv("PPE_CUT_LINES");
    const bool lines = lenv && *lenv ? *lenv == '1' : !lds_fit;
    // layout (ppe_image.h): header, bucket-length slices, group bases, fingerprints (what a lookup reads from LDS
    // when only they are staged), then the entries and ids
    const uint32_t off_cut = have_cut ? (end_tree + 7u) & ~7u : 0u;
    const uint32_t n_groups = have_cut ? std::max(1u, (1u << (cut.b0 + cut.b1)) / 32u) : 0u;
    const uint32_t n_ent = have_cut ? (uint32_t)cut.entries.size() : 0u;
    const uint32_t off_slc = off_cut + PPE_CUT_HDR_WORDS;                // 16 B per group, 16-B aligned
    const uint32_t off_gbase = off_slc + 4u * n_groups;                  // 4 B per group
    const uint32_t off_fp = off_gbase + n_groups;                        // 4 bits per entry (+ 2 pad words)
    // 128-B entry lines: epl 16-B entries, then (lines) their ids: 7 + 7 x 16 bit, or 6 + 6 x 32 bit; dense: 8
    // entries, the ids after the last line
    const uint32_t epl = !lines ? 8u : ids16 ? 7u : 6u;
    const uint32_t off_ent = (off_fp + (n_ent + 7u) / 8u + 2u + 31u) & ~31u;  // 128-B aligned
    const uint32_t n_lines = (n_ent + epl - 1u) / epl;
    const uint32_t off_id = lines ? 0u : off_ent + PPE_CUT_LINE_WORDS * n_lines;
    const uint32_t id_words = lines ? 0u : ids16 ? (n_ent + 1u) / 2u : n_ent;
    const uint32_t total = have_cut ? off_ent + PPE_CUT_LINE_WORDS * n_lines + id_words : end_tree;

    uint32_t *img = (uint32_t *)std::calloc(total, sizeof(uint32_t));
    if (!img) return PPE_ENOMEM;
    img[0] = PPE_IMG_MAGIC;
    img[1] = PPE_IMG_VERSION;
    img[PPE_IMG_W_NNODES] = n_nodes;
    img[PPE_IMG_W_NLEAF] = (uint32_t)leaf.size();
    img[PPE_IMG_W_NRULES] = n_slots;
    img[PPE_IMG_W_OFFNODES] = off_nodes;
    img[PPE_IMG_W_OFFLEAF] = off_leaf;
    img[PPE_IMG_W_OFFRULES] = off_rules;
    img[PPE_IMG_W_OFFRESID] = off_resid;
    img[PPE_IMG_W_DEFACT] = default_action;
    img[PPE_IMG_W_MAXDEPTH] = max_depth;
    img[PPE_IMG_W_MAXLEAF] = max_leaf;
    img[PPE_IMG_W_TOTAL] = total;
    img[PPE_IMG_W_ROOTKS] = nodes[0].dim << 8;
    img[PPE_IMG_W_JUMP] = jbest.bits ? (jbest.dim | (jbest.shift << 8) | (jbest.bits << 16)) : 0u;
    img[PPE_IMG_W_OFFBSEC] = off_bsec;
    img[PPE_IMG_W_NBLOCKS] = n_blocks;
    img[PPE_IMG_W_OFFBLOCKS] = off_blocks;
    img[PPE_IMG_W_MAXBDEPTH] = max_bdepth;
    img[PPE_IMG_W_OFFCREC] = off_crec;
    img[PPE_IMG_W_OFFIDTAB] = off_idtab;
    img[PPE_IMG_W_BLKLV] = 2u;
    img[PPE_IMG_W_OFFCUT] = off_cut;
    if (have_cut) {
        uint32_t *h = img + off_cut;
        h[0] = cut.b0 | (cut.b1 << 8) | (ids16 ? PPE_CUT_IDS16 : 0u) | (lines ? PPE_CUT_LINES : 0u);
        h[1] = 1u << (cut.b0 + cut.b1);
        h[2] = n_ent;
        h[3] = cut.max_len;
        h[4] = off_slc;
        h[5] = off_ent;
        h[6] = n_groups;
        h[7] = epl;
        h[8] = off_gbase;
        h[9] = off_fp;
        h[10] = epl == 8u ? 0x20000000u : epl == 7u ? 0x24924925u : 0x2AAAAAABu;  // e / epl = umulhi(e, h[10]), e < 2^25
        h[11] = n_lines;
        h[12] = off_id;
        const uint32_t nb = h[1];
        uint32_t first = 0;
        for (uint32_t g = 0; g < n_groups; ++g) {  // the group's first entry, its 32 lengths bit-sliced
            img[off_gbase + g] = first;
            uint32_t *sl = img + off_slc + 4u * g;
            for (uint32_t k = 0; k < 32u && 32u * g + k < nb; ++k) {
                const uint32_t len = cut.len[32u * g + k];
                for (uint32_t b = 0; b < 4u; ++b) sl[b] |= ((len >> b) & 1u) << k;
                first += len;
            }
        }
        // an address prefix relative to its bucket (ppe_image.h): the bits below the cut's b top bits shifted to the
        // top, their end marked by the next bit; a prefix no longer than b matches the whole bucket (marker bit 31)
        auto plen = [](uint32_t lo, uint32_t hi) { return 32u - (uint32_t)__builtin_popcount(hi - lo); };
        auto rel = [&](uint32_t lo, uint32_t hi, uint32_t b) -> uint32_t {
            const uint32_t len = plen(lo, hi);  // (hi - lo = 2^(32 - len) - 1)
            if (len <= b) return 0x80000000u;
            return (lo << b) | (1u << (31u - (len - b)));
        };
        uint8_t *fp = (uint8_t *)(img + off_fp);
        for (uint32_t e = 0; e < n_ent; ++e) {
            const Rule &r = R[cut.entries[e]];
            uint32_t *line = img + off_ent + PPE_CUT_LINE_WORDS * (e / epl);
            uint32_t *o = line + PPE_CUT_ENT_WORDS * (e % epl);
            const bool tcp = r.lo[PPE_DIM_PROTO] <= 6u && 6u <= r.hi[PPE_DIM_PROTO];
            const bool udp = r.lo[PPE_DIM_PROTO] <= 17u && 17u <= r.hi[PPE_DIM_PROTO];
            const bool drop = r.action == ACL_RULE_ACTION_DROP;
            o[0] = rel(r.lo[PPE_DIM_SIP], r.hi[PPE_DIM_SIP], cut.b0) | (drop ? 2u : 0u) | (tcp ? 1u : 0u);
            o[1] = rel(r.lo[PPE_DIM_DIP], r.hi[PPE_DIM_DIP], cut.b1) | (udp ? 1u : 0u);
            o[2] = r.lo[PPE_DIM_SPORT] | (r.lo[PPE_DIM_DPORT] << 16);
            o[3] = (r.hi[PPE_DIM_SPORT] - r.lo[PPE_DIM_SPORT]) | ((r.hi[PPE_DIM_DPORT] - r.lo[PPE_DIM_DPORT]) << 16);
            uint32_t *ids = lines ? line + PPE_CUT_ENT_WORDS * epl : img + off_id;
            const uint32_t k = lines ? e % epl : e;
            if (ids16) ((uint16_t *)ids)[k] = (uint16_t)r.id;
            else ids[k] = r.id;
            // fingerprint: the first sip / dip bit below the cut, each with its "the prefix fixes it" flag
            const bool sv = plen(r.lo[PPE_DIM_SIP], r.hi[PPE_DIM_SIP]) > cut.b0;
            const bool dv = plen(r.lo[PPE_DIM_DIP], r.hi[PPE_DIM_DIP]) > cut.b1;
            const uint32_t f = (sv ? ((r.lo[PPE_DIM_SIP] >> (31u - cut.b0)) & 1u) | 2u : 0u) |
                               (dv ? (((r.lo[PPE_DIM_DIP] >> (31u - cut.b1)) & 1u) << 2) | 8u : 0u);
            fp[e >> 1] |= (uint8_t)(f << (4u * (e & 1u)));
        }
    }
    if (compact) {
        // prefix | marker bit (len 0..31), or the address of a /32
        // (a prefix box spans 2^(32 - len) keys: its marker bit 1 << (31 - len) is half that count)
        auto pfx = [](uint32_t lo, uint32_t hi) { return lo == hi ? lo : lo | (((hi - lo) >> 1) + 1u); };
        for (uint32_t sl = 0; sl <= n_slots; ++sl) {
            uint32_t *o = img + off_crec + PPE_CREC_WORDS * sl;
            if (sl == n_slots) {  // sentinel: /0 addresses, every port
                o[0] = o[1] = 0x80000000u;
                o[2] = 0;
                o[3] = 0xffffffffu;
                continue;
            }
            const Rule &r = R[sl];
            o[0] = pfx(r.lo[PPE_DIM_SIP], r.hi[PPE_DIM_SIP]);
            o[1] = pfx(r.lo[PPE_DIM_DIP], r.hi[PPE_DIM_DIP]);
            o[2] = r.lo[PPE_DIM_SPORT] | (r.lo[PPE_DIM_DPORT] << 16);
            o[3] = (r.hi[PPE_DIM_SPORT] - r.lo[PPE_DIM_SPORT]) | ((r.hi[PPE_DIM_DPORT] - r.lo[PPE_DIM_DPORT]) << 16);
        }
        if (off_idtab) {
            for (uint32_t sl = 0; sl < n_slots; ++sl) img[off_idtab + sl] = R[sl].id;
            img[off_idtab + n_slots] = 0xffffffffu;  // the sentinel (its hit is -1 by its NOHIT flag)
        }
    }
    auto node_byte = [&](uint32_t k) { return 4u * off_nodes + 16u * k; };
    for (uint32_t k = 0; k < n_nodes; ++k) {
        const TNode &nd = nodes[k];
        uint32_t *o = img + off_nodes + PPE_NODE_WORDS * k;
        if (nd.dim == PPE_NODE_LEAF) {
            o[0] = PPE_LEAF_THR;
            o[1] = node_byte(k);
            if (max_leaf > 1)
                o[2] = nd.first | (std::min(nd.cnt, PPE_LEAF_CNT_ESC) << 24);
            else
                o[2] = nd.cnt ? leaf[nd.first] : n_slots;  // the sentinel slot for an empty leaf
            o[3] = (PPE_NODE_LEAF << 8) | (PPE_NODE_LEAF << 24);
        } else {
            o[0] = nd.thr;
            o[1] = node_byte(nd.left);
            o[2] = node_byte(nd.left + 1);
            o[3] = (nodes[nd.left].dim << 8) | (nodes[nd.left + 1].dim << 24);
        }
    }
    if (n_jump) {  // bucket → its subtree root: node byte offset | the root's key slot << 24; root block index
        uint32_t b = 0;
        for (uint32_t r = 0; r < best.n_roots; ++r)
            for (uint32_t i = 0; i < best.runs[r]; ++i, ++b) {
                img[PPE_IMG_HDR_WORDS + b] = node_byte(r) | (nodes[r].dim << 24);
                img[off_bsec + b] = r;  // root r's block is block r (the roots are the first blocks)
            }
    }
    std::memcpy(img + off_blocks, bwords.data(), bwords.size() * sizeof(uint32_t));
    if (!lwords.empty()) std::memcpy(img + off_leaf, lwords.data(), lwords.size() * sizeof(uint32_t));
    for (uint32_t s = 0; s <= n_slots; ++s) {
        uint32_t *o = img + off_rules + 8 * s;
        if (s == n_slots) {  // sentinel: matches every key, rule index -1, the default action
            o[0] = 0;
            o[1] = 0xffffffffu;
            o[2] = 0;
            o[3] = 0xffffffffu;
            o[4] = 0;
            o[5] = 0xffffffffu;
            o[6] = 0xffu << 8 | ((default_action & 0xffffu) << 16);
            o[7] = 0x1fffffffu;
            continue;
        }
        const Rule &r = R[s];
        o[0] = r.lo[PPE_DIM_SIP];
        o[1] = r.hi[PPE_DIM_SIP] - r.lo[PPE_DIM_SIP];
        o[2] = r.lo[PPE_DIM_DIP];
        o[3] = r.hi[PPE_DIM_DIP] - r.lo[PPE_DIM_DIP];
        o[4] = r.lo[PPE_DIM_SPORT] | (r.lo[PPE_DIM_DPORT] << 16);
        o[5] = (r.hi[PPE_DIM_SPORT] - r.lo[PPE_DIM_SPORT]) | ((r.hi[PPE_DIM_DPORT] - r.lo[PPE_DIM_DPORT]) << 16);
        o[6] = r.lo[PPE_DIM_PROTO] | ((r.hi[PPE_DIM_PROTO] - r.lo[PPE_DIM_PROTO]) << 8) | ((r.action & 0xffffu) << 16);
        o[7] = r.id | (r.resid << 29);
    }
    if (any_resid) std::memcpy(img + off_resid, resid_words.data(), resid_words.size() * sizeof(uint32_t));

    *words_out = img;
    *n_words_out = total;
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->n_rules = (uint32_t)R.size();
        st->n_nodes = n_nodes;
        st->n_leaves = n_leaves;
        st->n_leaf_entries = (uint32_t)leaf.size();
        st->max_depth = max_depth;
        st->avg_depth = n_leaves ? depth_sum / n_leaves : 0.0;
        st->blob_bytes = total * 4u;
        st->cut_bits = have_cut ? cut.b0 | (cut.b1 << 8) : 0u;
        st->cut_entries = have_cut ? (uint32_t)cut.entries.size() : 0u;
        st->build_ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return PPE_OK;
}

extern "C" void ppe_acl_free_image(uint32_t *words) { std::free(words); }
