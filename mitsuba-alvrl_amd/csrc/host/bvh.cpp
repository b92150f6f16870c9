// bvh.cpp -- host construction of the occluder BVH (see bvh.hpp).
#include "bvh.hpp"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace alvrl {

BvhHost build_bvh(const float* tri, uint32_t ntri, const uint32_t* material)
{
    BvhHost b;
    if (ntri == 0) return b;
    std::vector<uint32_t> idx(ntri);
    std::vector<float> cen(3 * (size_t)ntri);
    for (uint32_t i = 0; i < ntri; i++) {
        idx[i] = i;
        for (int a = 0; a < 3; a++)
            cen[3 * (size_t)i + a] = (tri[9 * (size_t)i + a] + tri[9 * (size_t)i + 3 + a] + tri[9 * (size_t)i + 6 + a]) * (1.0f / 3.0f);
    }
    struct Task { uint32_t node, begin, end, depth; };
    b.nodes.push_back(BvhNode{});
    std::vector<Task> stack{{0u, 0u, ntri, 0u}};
    while (!stack.empty()) {
        const Task t = stack.back();
        stack.pop_back();
        if (t.depth > kBvhMaxDepth) throw std::length_error("occluder BVH deeper than the traversal stack");
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t k = t.begin; k < t.end; k++) {
            const float* q = tri + 9 * (size_t)idx[k];
            for (int v = 0; v < 3; v++)
                for (int a = 0; a < 3; a++) {
                    lo[a] = std::min(lo[a], q[3 * v + a]);
                    hi[a] = std::max(hi[a], q[3 * v + a]);
                }
            for (int a = 0; a < 3; a++) {
                clo[a] = std::min(clo[a], cen[3 * (size_t)idx[k] + a]);
                chi[a] = std::max(chi[a], cen[3 * (size_t)idx[k] + a]);
            }
        }
        BvhNode& nd = b.nodes[t.node];
        for (int a = 0; a < 3; a++) {
            // conservative padding: the slab test's rounding stays inside it
            const float mag = std::max(std::fabs(lo[a]), std::fabs(hi[a]));
            const float pad = (hi[a] - lo[a]) * 1e-4f + 1e-5f * (1.0f + mag);
            nd.lo[a] = lo[a] - pad;
            nd.hi[a] = hi[a] + pad;
        }
        const uint32_t cnt = t.end - t.begin;
        if (cnt <= 4) {
            nd.a = (uint32_t)b.ids.size();
            nd.n = cnt;
            for (uint32_t k = t.begin; k < t.end; k++) {
                b.ids.push_back(idx[k] | (material && material[idx[k]] == 2u ? kBvhPassBit : 0u));
                b.tris.insert(b.tris.end(), tri + 9 * (size_t)idx[k], tri + 9 * (size_t)idx[k] + 9);
            }
            continue;
        }
        int ax = 0;
        for (int a = 1; a < 3; a++)
            if (chi[a] - clo[a] > chi[ax] - clo[ax]) ax = a;
        const uint32_t mid = t.begin + cnt / 2;
        std::nth_element(idx.begin() + t.begin, idx.begin() + mid, idx.begin() + t.end, [&](uint32_t x, uint32_t y) {
            const float cx = cen[3 * (size_t)x + ax], cy = cen[3 * (size_t)y + ax];
            return cx < cy || (cx == cy && x < y);
        });
        const uint32_t left = (uint32_t)b.nodes.size();
        b.nodes.push_back(BvhNode{});
        b.nodes.push_back(BvhNode{});
        b.nodes[t.node].a = left;   // (nd may dangle after the push_backs)
        b.nodes[t.node].n = 0;
        stack.push_back(Task{left + 1, mid, t.end, t.depth + 1});
        stack.push_back(Task{left, t.begin, mid, t.depth + 1});
    }
    return b;
}

}  // namespace alvrl
