// bvh_device.hpp -- occluder queries on the device: TriangleT::rayIntersect
// (include/mitsuba/core/triangle.h:109-145) over the host-built BVH
// (host/bvh.hpp).  Closest hit for eye rays and particles (Scene::rayIntersect:
// the shape kd-tree accepts t in [mint, maxt], skdtree.h:248-262) and any hit
// on a segment for the shadow tests of Scene::evalTransmittance
// (scene.cpp:619-679).
//
// The triangle test has the host's operation order (csrc/host/scene.cpp
// tri_intersect); in translation units built with -ffp-contract=off and IEEE
// division (tracer.hip) it returns the host's t bit for bit, and the closest
// hit takes the smallest t, ties to the lowest triangle index, which is what
// the host's loop in index order finds.  Traversal: a per-lane stack, the
// nearer child first; a node is skipped only if its (padded) slab interval
// misses [mint, best] -- a node at exactly the best t is still visited so
// that ties resolve by index.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "host/bvh.hpp"

namespace alvrl {
namespace bvh {

struct View {
    const BvhNode* nodes;
    const float* tris;      // 9 floats per leaf slot
    const uint32_t* ids;    // original triangle index per leaf slot
    uint32_t ntri;
};

struct V { float x, y, z; };
__device__ __forceinline__ V mk(float x, float y, float z) { return V{x, y, z}; }
__device__ __forceinline__ V sub(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V cross(V a, V b)
{
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

__device__ __forceinline__ bool tri_intersect(const float* q, V o, V d, float* u, float* v, float* t)
{
    const V p0 = mk(q[0], q[1], q[2]), p1 = mk(q[3], q[4], q[5]), p2 = mk(q[6], q[7], q[8]);
    const V edge1 = sub(p1, p0), edge2 = sub(p2, p0);
    const V pvec = cross(d, edge2);
    const float det = dot(edge1, pvec);
    if (det == 0) return false;
    const float inv_det = 1.0f / det;
    const V tvec = sub(o, p0);
    *u = dot(tvec, pvec) * inv_det;
    if (*u < 0.0f || *u > 1.0f) return false;
    const V qvec = cross(tvec, edge1);
    *v = dot(d, qvec) * inv_det;
    if (*v >= 0.0f && *u + *v <= 1.0f) {
        *t = dot(edge2, qvec) * inv_det;
        return true;
    }
    return false;
}

// slab interval of a padded node box intersected with [tmin, tmax]
__device__ __forceinline__ bool slab(const BvhNode& nd, V o, V inv, float tmin, float tmax, float* tnear)
{
    const float tx0 = (nd.lo[0] - o.x) * inv.x, tx1 = (nd.hi[0] - o.x) * inv.x;
    const float ty0 = (nd.lo[1] - o.y) * inv.y, ty1 = (nd.hi[1] - o.y) * inv.y;
    const float tz0 = (nd.lo[2] - o.z) * inv.z, tz1 = (nd.hi[2] - o.z) * inv.z;
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
    *tnear = tn;
    return tn <= tf;
}

__device__ __forceinline__ V inv_dir(V d)
{
    // a zero component: a huge finite slope keeps (lo - o) * inv ordered
    return mk(d.x != 0.0f ? 1.0f / d.x : copysignf(1e30f, d.x), d.y != 0.0f ? 1.0f / d.y : copysignf(1e30f, d.y),
              d.z != 0.0f ? 1.0f / d.z : copysignf(1e30f, d.z));
}

constexpr int kStack = 48;
static_assert(kBvhMaxDepth + 2 <= (uint32_t)kStack, "BVH depth cap vs traversal stack");

// Closest triangle hit with t in [mint, *best] that beats *best (strictly, or
// equal with a lower index than *best_id when *best_id >= 0).  Updates best,
// best_id (original index), slot (leaf slot, for the vertices), bu, bv.
__device__ inline void closest(const View& b, V o, V d, float mint, float* best, int* best_id, int* slot,
                               float* bu, float* bv)
{
    if (b.ntri == 0) return;
    const V inv = inv_dir(d);
    uint32_t stack[kStack];
    int sp = 0;
    stack[sp++] = 0u;
    while (sp > 0) {
        const BvhNode nd = b.nodes[stack[--sp]];
        float tn;
        if (!slab(nd, o, inv, mint, *best, &tn)) continue;
        if (nd.n > 0) {
            for (uint32_t k = nd.a; k < nd.a + nd.n; k++) {
                float u, v, t;
                if (!tri_intersect(b.tris + 9 * (size_t)k, o, d, &u, &v, &t)) continue;
                if (t < mint) continue;
                const int id = (int)(b.ids[k] & ~kBvhPassBit);
                if (t < *best || (t == *best && *best_id >= 0 && id < *best_id)) {
                    *best = t; *best_id = id; *slot = (int)k; *bu = u; *bv = v;
                }
            }
        } else {   // the build caps the depth (kBvhMaxDepth), so the stack never overflows
            float t0, t1;
            const bool h0 = slab(b.nodes[nd.a], o, inv, mint, *best, &t0);
            const bool h1 = slab(b.nodes[nd.a + 1], o, inv, mint, *best, &t1);
            if (h0 && h1) {
                // push the farther first: the nearer is popped next
                if (t0 <= t1) { stack[sp++] = nd.a + 1; stack[sp++] = nd.a; }
                else { stack[sp++] = nd.a; stack[sp++] = nd.a + 1; }
            } else if (h0) {
                stack[sp++] = nd.a;
            } else if (h1) {
                stack[sp++] = nd.a + 1;
            }
        }
    }
}

// Any triangle hit with t in [mint, maxt] (the occluder test of
// evalTransmittance on the segment p1 -> p1 + maxt * d).
__device__ inline bool occluded(const View& b, V o, V d, float mint, float maxt)
{
    if (b.ntri == 0) return false;
    const V inv = inv_dir(d);
    uint32_t stack[kStack];
    int sp = 0;
    stack[sp++] = 0u;
    while (sp > 0) {
        const BvhNode nd = b.nodes[stack[--sp]];
        float tn;
        if (!slab(nd, o, inv, mint, maxt, &tn)) continue;
        if (nd.n > 0) {
            for (uint32_t k = nd.a; k < nd.a + nd.n; k++) {
                if (b.ids[k] & kBvhPassBit) continue;   // a null-BSDF surface lets the segment pass
                float u, v, t;
                if (tri_intersect(b.tris + 9 * (size_t)k, o, d, &u, &v, &t) && !(t < mint || t > maxt)) return true;
            }
        } else {
            stack[sp++] = nd.a + 1;
            stack[sp++] = nd.a;
        }
    }
    return false;
}

}  // namespace bvh
}  // namespace alvrl
