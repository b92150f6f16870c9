// preprocessor.hpp -- host part of LightSlice (Preprocessor.cpp): slicing,
// representative pixels, localities and local-matrix rows.  The matrix work
// (R build, clustering refinement) runs on the device through include/alvrl.h.
#pragma once

#include <cstdint>
#include <set>
#include <utility>
#include <vector>

#include "scene.hpp"

namespace alvrl {
namespace host {

struct PrepParams {
    uint32_t target_num_slices = 100;   // targetNumSlices
    uint32_t neighbour_count = 0;       // neighbourCount
    float neighbour_weight = 0.0f;      // neighbourWeight
    float slice_curvature_factor = 0.5f;// sliceCurvatureFactor
    uint32_t seed = 0, pass = 0;
};

class Preprocessor {
public:
    explicit Preprocessor(const PrepParams& p) : m_p(p) {}

    // buildSlices (Preprocessor.cpp:1130-1193) + getSlices / getSlicesPQ
    // (:1200-1418).  Returns the pixel -> slice map indexed y + H*x.
    // recs: the W*H gather records in row-major pixel order (the GPU eye-ray
    // first hits, alvrl_scene_records_gpu), or null to form them here
    std::vector<uint32_t> build_slices(const SmokeBox& s, const float* recs = nullptr);
    // sampleSliceMapping (:1502-1525): representative pixels per slice (pixel
    // ids in the column-major numbering x*H + y), m_sliceUndersampling,
    // buildLocalities (:1241-1293) and m_globalPixelUndersampling.
    void sample_slice_mapping(float target_pixel_undersampling);
    // getLocalMatrix (:779-827): local rows (global row ids, rows are the
    // representatives in slice-major order) and locality weights.
    void local_matrix(uint32_t slice, std::vector<uint32_t>* rows, std::vector<double>* w) const;

    void set_pass(uint32_t pass) { m_p.pass = pass; }
    uint32_t num_slices() const { return (uint32_t)m_lo.size(); }
    const std::vector<uint32_t>& rep_off() const { return m_rep_off; }
    const std::vector<uint32_t>& rep_pix() const { return m_rep_pix; }
    const std::vector<float>& slice_undersampling() const { return m_slice_under; }
    float global_pixel_undersampling() const { return m_global_under; }
    uint32_t slice_pixels(uint32_t s) const { return m_hi[s] - m_lo[s]; }

private:
    PrepParams m_p;
    int m_W = 0, m_H = 0;
    std::vector<uint32_t> m_idx;            // gather point ids, partitioned by slice
    std::vector<uint32_t> m_lo, m_hi;       // slice s = m_idx[m_lo[s] .. m_hi[s])
    std::vector<V3> m_posC, m_dirC;         // slice centroids
    std::vector<uint32_t> m_rep_off, m_rep_pix;
    std::vector<float> m_slice_under;
    float m_global_under = -1.0f;
    std::vector<std::set<std::pair<uint32_t, float>>> m_loc;
};

}  // namespace host
}  // namespace alvrl
