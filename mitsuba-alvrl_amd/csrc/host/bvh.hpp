// bvh.hpp -- bounding-volume hierarchy over the occluder triangles of a
// scene (the MI355X stand-in for Mitsuba's ShapeKDTree, skdtree.h, which
// answers Scene::rayIntersect and the occlusion part of evalTransmittance).
// Built on the host, traversed on the device (bvh_device.hpp) by the eye-ray
// kernel, the GPU tracer and the gathers' shadow tests.  Node bounds are
// padded so that the float slab test never rejects a box whose triangles the
// exact triangle test would accept; the triangle test itself is
// TriangleT::rayIntersect (include/mitsuba/core/triangle.h:109-145) in the
// host's operation order, so a closest hit through the BVH equals the host's
// brute-force loop (same t, ties to the lowest triangle index).
#pragma once

#include <cstdint>
#include <vector>

namespace alvrl {

// 32 bytes.  n > 0: leaf over triangles [a, a + n) of the reordered arrays;
// n == 0: inner node with children a and a + 1.
struct BvhNode {
    float lo[3];
    uint32_t a;
    float hi[3];
    uint32_t n;
};
static_assert(sizeof(BvhNode) == 32, "BvhNode layout");

struct BvhHost {
    std::vector<BvhNode> nodes;     // root = nodes[0]
    std::vector<float> tris;        // 9 floats per triangle, leaf order
    std::vector<uint32_t> ids;      // original triangle index per leaf slot (| kBvhPassBit)
};

// ids bit 31: a null-BSDF triangle, which the occlusion test passes
// (Scene::evalTransmittance, scene.cpp:636-637) but closest hits see
constexpr uint32_t kBvhPassBit = 0x80000000u;
constexpr uint32_t kBvhMaxDepth = 40;   // the traversal stacks hold 48 nodes

// Median split on the widest centroid axis (ties by triangle index), leaves
// of at most 4 triangles; deterministic.  material: per triangle (2 = null:
// kBvhPassBit), or null.  Throws std::length_error if the tree would be
// deeper than kBvhMaxDepth (the device traversal could not hold it).
BvhHost build_bvh(const float* tri, uint32_t ntri, const uint32_t* material = nullptr);

}  // namespace alvrl
