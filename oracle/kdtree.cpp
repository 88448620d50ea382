// TEST INFRASTRUCTURE ONLY -- exact k-NN used by the CPU restatement.
//
// Stands in for PCL KdTreeFLANN (external: PCL >= 1.7, FLANN 1.8.x inferred; call sites
// REG/FeatureMatch/FeatureMatchBase.hpp:36,42, EdgeFeatureMatch.hpp:38, surfFeatureMatch.hpp:37).
// Published FLANN semantics restated: single kd-tree, max leaf size 15, middle split on the
// widest dimension, exact search (eps = 0), results sorted ascending, L2_Simple float distance
// ((0 + dx^2) + dy^2) + dz^2.  FLANN leaves equal-distance order unspecified; here ties are
// broken by ascending map index (the canonical rule shared with the GPU path).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "lmsf_oracle.h"


namespace {

constexpr int kLeaf = 15;

struct Node {
    int dim;          // -1 for a leaf
    float split;
    int left, right;  // child node ids
    int begin, end;   // leaf range into perm
    float lo[3], hi[3];
};

struct Key {
    float d2;
    int32_t idx;
};
inline bool key_less(const Key& a, const Key& b) {
    return a.d2 < b.d2 || (a.d2 == b.d2 && a.idx < b.idx);
}

}  // namespace

struct lmsfo_map {
    std::vector<float> xyz;     // 3 per point, original order
    std::vector<int32_t> perm;  // leaf order
    std::vector<Node> nodes;
    int64_t n = 0;

    int build(int begin, int end, int depth) {
        Node nd;
        for (int d = 0; d < 3; ++d) {
            nd.lo[d] = std::numeric_limits<float>::infinity();
            nd.hi[d] = -std::numeric_limits<float>::infinity();
        }
        for (int i = begin; i < end; ++i) {
            const float* p = &xyz[3 * (size_t)perm[i]];
            for (int d = 0; d < 3; ++d) {
                nd.lo[d] = std::min(nd.lo[d], p[d]);
                nd.hi[d] = std::max(nd.hi[d], p[d]);
            }
        }
        nd.begin = begin;
        nd.end = end;
        nd.left = nd.right = -1;
        nd.dim = -1;
        nd.split = 0.f;
        int id = (int)nodes.size();
        nodes.push_back(nd);
        if (end - begin <= kLeaf) return id;
        int dim = 0;
        float span = nd.hi[0] - nd.lo[0];
        for (int d = 1; d < 3; ++d)
            if (nd.hi[d] - nd.lo[d] > span) { span = nd.hi[d] - nd.lo[d]; dim = d; }
        if (!(span > 0.f)) return id;  // all points identical: keep as a (large) leaf
        float split = 0.5f * (nd.lo[dim] + nd.hi[dim]);
        int mid = begin;
        if (depth < 48) {
            auto mid_it = std::partition(perm.begin() + begin, perm.begin() + end,
                                         [&](int32_t k) { return xyz[3 * (size_t)k + dim] < split; });
            mid = (int)(mid_it - perm.begin());
        }
        // degenerate middle split (or a deep tree) -> median split; keeps depth <= 48 + log2(n)
        if (mid == begin || mid == end) {
            mid = begin + (end - begin) / 2;
            std::nth_element(perm.begin() + begin, perm.begin() + mid, perm.begin() + end,
                             [&](int32_t a, int32_t b) { return xyz[3 * (size_t)a + dim] < xyz[3 * (size_t)b + dim]; });
            split = xyz[3 * (size_t)perm[mid] + dim];
        }
        int l = build(begin, mid, depth + 1);
        int r = build(mid, end, depth + 1);
        nodes[id].dim = dim;
        nodes[id].split = split;
        nodes[id].left = l;
        nodes[id].right = r;
        return id;
    }

    // squared float distance from q to the node's bounding box (lower bound, computed with a
    // relative slack so float rounding can never prune a point whose computed distance ties)
    static float box_d2(const Node& nd, const float* q) {
        float s = 0.f;
        for (int d = 0; d < 3; ++d) {
            float v = 0.f;
            if (q[d] < nd.lo[d]) v = nd.lo[d] - q[d];
            else if (q[d] > nd.hi[d]) v = q[d] - nd.hi[d];
            s += v * v;
        }
        return s;
    }

    void knn(const float* q, int k, Key* best) const {
        for (int i = 0; i < k; ++i) best[i] = {std::numeric_limits<float>::infinity(), INT32_MAX};
        if (nodes.empty()) return;
        // a non-finite query (a NaN pose) has a NaN or +inf distance to every point: no key is ever less than
        // the empty slots, and box_d2's NaN would walk the whole tree to find that out
        if (!(std::isfinite(q[0]) && std::isfinite(q[1]) && std::isfinite(q[2]))) return;
        int stack[128];
        int sp = 0;
        stack[sp++] = 0;
        while (sp > 0) {
            const Node& nd = nodes[stack[--sp]];
            float lb = box_d2(nd, q);
            if (lb > best[k - 1].d2 * (1.0f + 1e-6f)) continue;
            if (nd.dim < 0) {
                for (int i = nd.begin; i < nd.end; ++i) {
                    int32_t pi = perm[i];
                    const float* p = &xyz[3 * (size_t)pi];
                    float dx = q[0] - p[0];
                    float dy = q[1] - p[1];
                    float dz = q[2] - p[2];
                    float d2 = dx * dx + dy * dy + dz * dz;
                    Key key{d2, pi};
                    if (key_less(key, best[k - 1])) {
                        int j = k - 1;
                        while (j > 0 && key_less(key, best[j - 1])) { best[j] = best[j - 1]; --j; }
                        best[j] = key;
                    }
                }
                continue;
            }
            // push far child first so the near child is visited first
            float diff = q[nd.dim] - nd.split;
            int near = diff < 0 ? nd.left : nd.right;
            int far = diff < 0 ? nd.right : nd.left;
            stack[sp++] = far;
            stack[sp++] = near;
        }
    }
};

extern "C" lmsfo_map* lmsfo_map_build(const float* xyzi, int64_t n) {
    lmsfo_map* m = new lmsfo_map();
    m->n = n;
    m->xyz.resize(3 * (size_t)n);
    m->perm.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        m->xyz[3 * i + 0] = xyzi[4 * i + 0];
        m->xyz[3 * i + 1] = xyzi[4 * i + 1];
        m->xyz[3 * i + 2] = xyzi[4 * i + 2];
        m->perm[i] = (int32_t)i;
    }
    if (n > 0) m->build(0, (int)n, 0);
    return m;
}

extern "C" void lmsfo_map_free(lmsfo_map* m) { delete m; }
extern "C" int64_t lmsfo_map_size(const lmsfo_map* m) { return m ? m->n : 0; }

// Shared by the registration restatement.
void lmsfo_map_knn_one(const lmsfo_map* m, const float q[3], int k, int32_t* idx, float* d2) {
    Key best[16];
    m->knn(q, k, best);
    for (int i = 0; i < k; ++i) {
        bool ok = best[i].idx != INT32_MAX;
        idx[i] = ok ? best[i].idx : -1;
        d2[i] = ok ? best[i].d2 : std::numeric_limits<float>::infinity();
    }
}

extern "C" int lmsfo_map_knn(const lmsfo_map* m, const float* q, int64_t nq, int k, int32_t* idx, float* d2) {
    if (k < 1 || k > 16) return -1;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nq; ++i) lmsfo_map_knn_one(m, q + 4 * i, k, idx + k * i, d2 + k * i);
    return 0;
}

extern "C" int lmsfo_brute_knn(const float* map_xyzi, int64_t n, const float* q, int64_t nq, int k,
                               int32_t* idx, float* d2) {
    if (k < 1 || k > 16) return -1;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nq; ++i) {
        Key best[16];
        for (int j = 0; j < k; ++j) best[j] = {std::numeric_limits<float>::infinity(), INT32_MAX};
        const float* qq = q + 4 * i;
        for (int64_t p = 0; p < n; ++p) {
            float dx = qq[0] - map_xyzi[4 * p + 0];
            float dy = qq[1] - map_xyzi[4 * p + 1];
            float dz = qq[2] - map_xyzi[4 * p + 2];
            float dd = dx * dx + dy * dy + dz * dz;
            Key key{dd, (int32_t)p};
            if (key_less(key, best[k - 1])) {
                int j = k - 1;
                while (j > 0 && key_less(key, best[j - 1])) { best[j] = best[j - 1]; --j; }
                best[j] = key;
            }
        }
        for (int j = 0; j < k; ++j) {
            bool ok = best[j].idx != INT32_MAX;
            idx[k * i + j] = ok ? best[j].idx : -1;
            d2[k * i + j] = ok ? best[j].d2 : std::numeric_limits<float>::infinity();
        }
    }
    return 0;
}
