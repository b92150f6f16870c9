/*
 * vrlAmdIntegrator.cpp -- the "vrl_amd" Mitsuba integrator plugin: the vrl
 * integrator (src/integrators/vrl/vrlIntegrator.cpp) with its hot path --
 * the per-pixel VRL gather, the reduced matrix R and the per-slice cluster
 * refinement -- on an MI355X through libalvrl.so (include/alvrl.h,
 * include/alvrl_host.h).
 *
 * Build: compiled inside the mitsuba-ALVRL tree against its headers, like
 * the reference plugin (INTEGRATION.md "Build"); links libalvrl.so and the
 * HIP runtime.  This file is not compiled in this repository (no Mitsuba
 * headers or Boost here); tests/test_plugin_source.py checks that every
 * libalvrl entry point it calls is exported with the declared signature.
 *
 * Two modes, chosen by the property "amdMode":
 *
 *   "frame" (default)  The scene is described to the library once
 *                      (camera, film, the homogeneous medium's container
 *                      box and its diffuse walls, a point light, triangle
 *                      occluders with diffuse / mirror / null BSDFs).  The
 *                      library traces the VRLs, builds R, refines the
 *                      clusters and renders the whole frame on the GPU once
 *                      per pass; renderBlock copies its block out of that
 *                      frame.  Delta-BSDF chains are expanded by the library
 *                      (LiInternal's recursion, :445-511).
 *
 *   "records"          For scenes the descriptor cannot express: Mitsuba
 *                      itself casts the eye rays (and follows specular
 *                      chains) in renderBlock and hands the device one gather
 *                      record per eye segment (alvrl_gather_rec);
 *                      alvrl_gather_clustered_host / alvrl_gather_brute_host
 *                      return the radiance of each.  Worker threads call it
 *                      concurrently: the library gives every calling thread
 *                      its own HIP stream and scratch (alvrl.h "Threading").
 *                      The VRLs and the cluster lists still come from the
 *                      library's prepass over the descriptor's occluders,
 *                      so the scene's triangles are handed to it as
 *                      occluders for the gathers' visibility tests.
 *
 * Properties: every property of the reference integrator, with its name and
 * default (vrlIntegrator.cpp:128-208), is parsed by the library
 * (alvrl_integrator_create).  The homogeneous medium's sampling settings are
 * private to its plugin, so the scene file repeats them on the integrator
 * when they differ from the defaults: "mediumSamplingWeight", "strategy",
 * "channel", "samplingDensity" (homogeneous.cpp:156-227).
 */
#include <mitsuba/core/plugin.h>
#include <mitsuba/render/bsdf.h>
#include <mitsuba/render/emitter.h>
#include <mitsuba/render/medium.h>
#include <mitsuba/render/phase.h>
#include <mitsuba/render/scene.h>
#include <mitsuba/render/sensor.h>
#include <mitsuba/render/trimesh.h>

#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <mutex>
#include <sstream>
#include <vector>

#include "alvrl.h"
#include "alvrl_host.h"

MTS_NAMESPACE_BEGIN

namespace {

/* ALVRL_ERR_* -> Log(EError), which throws like the reference's own errors */
void check(int rc, const char *what) {
    if (rc != ALVRL_OK)
        SLog(EError, "vrl_amd: %s: %s", what, alvrl_host_last_error());
}
void checkDevice(int rc, alvrl_ctx *ctx, const char *what) {
    if (rc != ALVRL_OK)
        SLog(EError, "vrl_amd: %s: %s", what, alvrl_last_error(ctx));
}
void checkHip(hipError_t e, const char *what) {
    if (e != hipSuccess)
        SLog(EError, "vrl_amd: %s: %s", what, hipGetErrorString(e));
}

void put3(float *dst, const Spectrum &s) {
    Float r, g, b;
    s.toLinearRGB(r, g, b);
    dst[0] = (float) r; dst[1] = (float) g; dst[2] = (float) b;
}

/* The properties the library does not take (Mitsuba's own, or the medium's
 * restated on the integrator) */
bool isMitsubaOnly(const std::string &k) {
    return k == "amdMode" || k == "amdDevice" || k == "mediumSamplingWeight" || k == "strategy" ||
        k == "channel" || k == "samplingDensity";
}

} // namespace

class vrlAmdIntegrator : public ProgressiveMonteCarloIntegrator {
public:
    vrlAmdIntegrator(const Properties &props) : ProgressiveMonteCarloIntegrator(props) {
        m_recordsMode = props.getString("amdMode", "frame") == "records";
        if (!m_recordsMode && props.getString("amdMode", "frame") != "frame")
            Log(EError, "amdMode must be \"frame\" or \"records\"");
        m_device = props.getInteger("amdDevice", 0);
        m_samplingWeight = props.getFloat("mediumSamplingWeight", -1);
        std::string strategy = props.getString("strategy", "balance");
        if (strategy == "balance") m_strategy = ALVRL_STRATEGY_BALANCE;
        else if (strategy == "single") m_strategy = ALVRL_STRATEGY_SINGLE;
        else if (strategy == "manual") m_strategy = ALVRL_STRATEGY_MANUAL;
        else if (strategy == "maximum") m_strategy = ALVRL_STRATEGY_MAXIMUM;
        else Log(EError, "Specified an unknown sampling strategy");
        m_channel = props.getInteger("channel", -1) + 1;
        m_samplingDensity = props.getFloat("samplingDensity", 0.0f);
        m_specRRdepth = props.getInteger("specularForcedRRdepth", 100);
        m_initialSpecularThroughput = props.getFloat("initialSpecularThroughput", 20);

        std::vector<std::string> names;
        props.putPropertyNames(names);
        std::ostringstream oss;
        for (size_t i = 0; i < names.size(); ++i) {
            if (isMitsubaOnly(names[i]))
                continue;
            oss << names[i] << "=" << props.getAsString(names[i]) << ";";
        }
        m_props = oss.str();
        check(alvrl_integrator_create(m_props.c_str(), m_device, &m_it), "alvrl_integrator_create");
        checkHip(hipSetDevice(m_device), "hipSetDevice");
        checkHip(hipStreamCreateWithFlags(&m_stream, hipStreamNonBlocking), "hipStreamCreate");
    }

    ~vrlAmdIntegrator() {
        if (m_fb) hipFree(m_fb);
        if (m_stream) hipStreamDestroy(m_stream);
        alvrl_integrator_destroy(m_it);
    }

    bool preprocess(const Scene *scene, RenderQueue *queue, const RenderJob *job,
            int sceneResID, int sensorResID, int samplerResID) {
        ProgressiveMonteCarloIntegrator::preprocess(scene, queue, job, sceneResID,
            sensorResID, samplerResID);
        /* the sampler's sampleCount: sensor samples per pixel and pass
           (renderBlock's sample loop, integrator.cpp:240-264); the frame
           mode's integrator jitters them itself, so it is re-created with it */
        const Sampler *smp = static_cast<Sampler *>(Scheduler::getInstance()->getResource(samplerResID, 0));
        m_sampleCount = (int) smp->getSampleCount();
        if (!m_recordsMode && m_sampleCount != 1) {
            std::ostringstream oss;
            oss << m_props << "sampleCount=" << m_sampleCount << ";";
            alvrl_integrator_destroy(m_it);
            m_it = NULL;
            check(alvrl_integrator_create(oss.str().c_str(), m_device, &m_it), "alvrl_integrator_create");
        }
        describe(scene);
        alvrl_scene_desc sd = m_desc;
        sd.occluders = m_tris.empty() ? NULL : &m_tris[0];
        sd.occluder_material = m_mats.empty() ? NULL : &m_mats[0];
        check(alvrl_integrator_preprocess(m_it, &sd), "alvrl_integrator_preprocess");
        const Vector2i size = scene->getSensor()->getFilm()->getCropSize();
        m_width = size.x; m_height = size.y;
        m_rgb.assign((size_t) 3 * m_width * m_height, 0.0f);
        if (m_fb) hipFree(m_fb);
        checkHip(hipMalloc(&m_fb, sizeof(float) * m_rgb.size()), "hipMalloc");
        return true;
    }

    /* vrlIntegrator::prepass (:270-356): VRLs, representatives, R, clusters */
    bool prepass(const Scene *, Sampler *) {
        check(alvrl_integrator_prepass(m_it, m_pass), "alvrl_integrator_prepass");
        if (m_recordsMode) {   // the slice of every pixel, for the blocks' clustered gathers
            m_p2s.clear();
            if (alvrl_integrator_num_slices(m_it) > 0) {
                m_p2s.resize((size_t) m_width * m_height);
                check(alvrl_integrator_slices(m_it, &m_p2s[0], (uint32_t) m_p2s.size()), "alvrl_integrator_slices");
            }
        }
        std::lock_guard<std::mutex> g(m_frameLock);
        m_framePass = -1;   // the frame of the new pass is rendered on first use
        ++m_pass;
        return true;
    }

    void renderBlock(const Scene *scene, const Sensor *sensor, Sampler *sampler, ImageBlock *block,
            const bool &stop, const std::vector< TPoint2<uint8_t> > &points) const {
        block->clear();
        if (m_recordsMode) {
            renderBlockRecords(scene, sensor, sampler, block, stop, points);
            return;
        }
        ensureFrame();
        const Point2i off = block->getOffset();
        Float alpha = 1.0f;
        for (size_t i = 0; i < points.size() && !stop; ++i) {
            const Point2i p = Point2i(points[i]) + Vector2i(off);
            const float *c = &m_rgb[3 * ((size_t) p.y * m_width + p.x)];
            Spectrum s;
            s.fromLinearRGB(c[0], c[1], c[2]);
            block->put(Point2(p) + Vector2(0.5f), s, alpha);
        }
    }

    Spectrum Li(const RayDifferential &, RadianceQueryRecord &) const {
        Log(EError, "vrl_amd renders whole blocks (renderBlock)");
        return Spectrum(0.0f);
    }

    std::string passFileSuffix() {
        alvrl_integrator_stats st;
        check(alvrl_integrator_get_stats(m_it, &st), "alvrl_integrator_get_stats");
        std::ostringstream oss;
        oss << std::scientific << "_prevrl" << (double) st.contrib_preprocess
            << "_renvrl" << (double) st.contrib_render;
        return oss.str();
    }

    std::string toString() const {
        return std::string("vrlAmdIntegrator[mode=") + (m_recordsMode ? "records" : "frame") + "]";
    }

    MTS_DECLARE_CLASS()

private:
    /* The scene in the library's terms (alvrl_scene_desc): the perspective
     * camera, the medium and its container box, the point light, and the
     * remaining triangles as occluders. */
    void describe(const Scene *scene) {
        alvrl_scene_default(&m_desc, 1, 1);
        const Sensor *sensor = scene->getSensor();
        const PerspectiveCamera *cam = dynamic_cast<const PerspectiveCamera *>(sensor);
        if (!cam)
            Log(EError, "vrl_amd needs a perspective camera");
        const Transform toWorld = cam->getWorldTransform()->eval(0);
        const Point o = toWorld(Point(0.0f));
        const Point t = toWorld(Point(0.0f, 0.0f, 1.0f));
        const Vector up = toWorld(Vector(0.0f, 1.0f, 0.0f));
        for (int i = 0; i < 3; ++i) {
            m_desc.cam_origin[i] = (float) o[i];
            m_desc.cam_target[i] = (float) t[i];
            m_desc.cam_up[i] = (float) up[i];
        }
        m_desc.fov_x_deg = (float) cam->getXFov();
        const Vector2i size = sensor->getFilm()->getCropSize();
        m_desc.width = size.x; m_desc.height = size.y;

        /* the medium and the shape that contains it */
        const Medium *medium = sensor->getMedium();
        if (!medium || scene->getMedia().size() != 1)
            Log(EError, "vrl_amd needs the camera inside one homogeneous medium");
        const Spectrum ss = medium->getSigmaS(), sa = medium->getSigmaA();
        for (int i = 0; i < 3; ++i) {
            m_desc.medium.sigma_s[i] = (float) ss[i];
            m_desc.medium.sigma_a[i] = (float) sa[i];
        }
        m_desc.medium.sampling_weight = m_samplingWeight;
        m_desc.medium.strategy = m_strategy;
        m_desc.medium.channel = m_channel;
        m_desc.medium.sampling_density = m_samplingDensity;
        const PhaseFunction *phase = medium->getPhaseFunction();
        const bool hg = phase->getClass()->getName() == "HGPhaseFunction";
        m_desc.medium.phase_type = hg ? 1 : 0;
        m_desc.medium.phase_g = hg ? (float) phase->getMeanCosine() : 0.0f;

        /* the point light: samplePosition returns its power, intensity * 4 pi (point.cpp:81-91) */
        const Emitter *light = NULL;
        for (size_t i = 0; i < scene->getEmitters().size(); ++i)
            if (scene->getEmitters()[i]->getType() & Emitter::EDeltaPosition)
                light = scene->getEmitters()[i].get();
        if (!light)
            Log(EError, "vrl_amd needs a point light");
        PositionSamplingRecord pRec(0.0f);
        const Spectrum power = light->samplePosition(pRec, Point2(0.5f));
        put3(m_desc.light_intensity, power * (Float) (0.25f * INV_PI));
        for (int i = 0; i < 3; ++i) m_desc.light_pos[i] = (float) pRec.p[i];

        /* the container: the shape whose interior is the medium; its walls' diffuse reflectance */
        m_tris.clear(); m_mats.clear();
        bool haveBox = false, haveOccAlbedo = false, haveSpec = false;
        const ref_vector<Shape> &shapes = scene->getShapes();
        for (size_t s = 0; s < shapes.size(); ++s) {
            const Shape *sh = shapes[s].get();
            const BSDF *bsdf = sh->getBSDF();
            Intersection its;
            if (sh->getInteriorMedium() == medium && !haveBox) {
                const AABB box = sh->getAABB();
                for (int i = 0; i < 3; ++i) {
                    m_desc.box_min[i] = (float) box.min[i];
                    m_desc.box_max[i] = (float) box.max[i];
                }
                if (bsdf) put3(m_desc.albedo, bsdf->getDiffuseReflectance(its));
                haveBox = true;
                continue;
            }
            const TriMesh *mesh = dynamic_cast<const TriMesh *>(sh);
            if (!mesh)
                Log(EError, "vrl_amd: shape \"%s\" inside the medium is not a triangle mesh",
                    sh->getName().c_str());
            uint32_t mat = ALVRL_MAT_DIFFUSE;
            if (bsdf) {
                const unsigned int type = bsdf->getType();
                if (type & BSDF::ENull) {
                    mat = ALVRL_MAT_NULL;
                } else if ((type & BSDF::EDeltaReflection) && !(type & BSDF::ESmooth)) {
                    mat = ALVRL_MAT_MIRROR;
                    if (!haveSpec) put3(m_desc.occluder_specular, bsdf->getSpecularReflectance(its));
                    haveSpec = true;
                } else if (!haveOccAlbedo) {
                    put3(m_desc.occluder_albedo, bsdf->getDiffuseReflectance(its));
                    haveOccAlbedo = true;
                }
            }
            const Point *pos = mesh->getVertexPositions();
            const Triangle *tri = mesh->getTriangles();
            for (size_t f = 0; f < mesh->getTriangleCount(); ++f) {
                for (int k = 0; k < 3; ++k) {
                    const Point &p = pos[tri[f].idx[k]];
                    m_tris.push_back((float) p.x);
                    m_tris.push_back((float) p.y);
                    m_tris.push_back((float) p.z);
                }
                m_mats.push_back(mat);
            }
        }
        if (!haveBox)
            Log(EError, "vrl_amd needs a shape that contains the medium (its interior)");
        m_desc.n_occluders = (uint32_t) m_mats.size();
    }

    /* "frame" mode: one device render of the whole frame per pass, shared by
     * all blocks (the first block of a pass renders, the others wait) */
    void ensureFrame() const {
        std::unique_lock<std::mutex> g(m_frameLock);
        if (m_framePass == m_pass) return;
        if (m_rendering) {
            m_frameReady.wait(g, [this] { return !m_rendering; });
            if (m_framePass == m_pass) return;
        }
        m_rendering = true;
        g.unlock();
        int rc = ALVRL_OK;
        hipError_t e = hipSetDevice(m_device);
        if (e == hipSuccess) e = hipMemsetAsync(m_fb, 0, sizeof(float) * m_rgb.size(), m_stream);
        if (e == hipSuccess) rc = alvrl_integrator_render(m_it, 0, 1, m_fb, m_stream);
        if (e == hipSuccess && rc == ALVRL_OK)
            e = hipMemcpyAsync(&m_rgb[0], m_fb, sizeof(float) * m_rgb.size(), hipMemcpyDeviceToHost, m_stream);
        if (e == hipSuccess && rc == ALVRL_OK) e = hipStreamSynchronize(m_stream);
        g.lock();
        m_rendering = false;
        if (e == hipSuccess && rc == ALVRL_OK) m_framePass = m_pass;
        m_frameReady.notify_all();
        g.unlock();
        checkHip(e, "frame render");
        check(rc, "alvrl_integrator_render");
    }

    /* "records" mode: LiInternal's eye path per pixel (:398-524), cast by
     * Mitsuba; one record per segment with the recursion's weight */
    void renderBlockRecords(const Scene *scene, const Sensor *sensor, Sampler *sampler, ImageBlock *block,
            const bool &stop, const std::vector< TPoint2<uint8_t> > &points) const {
        alvrl_ctx *ctx = alvrl_integrator_ctx(m_it);
        const Point2i off = block->getOffset();
        std::vector<alvrl_gather_rec> recs;
        std::vector<uint32_t> ids, slice, owner;
        const bool clustered = !m_p2s.empty();
        std::vector<Point2> pos;   // each sensor sample's image position
        for (size_t i = 0; i < points.size() && !stop; ++i) {
          const Point2i p = Point2i(points[i]) + Vector2i(off);
          const uint32_t pid = (uint32_t) p.y * (uint32_t) m_width + (uint32_t) p.x;
          const uint32_t sl = clustered ? m_p2s[(size_t) p.y + (size_t) m_height * p.x] : 0u;   // m_slices[y + H*x]
          sampler->generate(p);
          for (size_t j = 0; j < sampler->getSampleCount(); ++j) {
            RadianceQueryRecord rRec(scene, sampler);
            rRec.newQuery(RadianceQueryRecord::ESensorRay, sensor->getMedium());
            /* the pixel centre for one sample per pixel, else a sampler draw (integrator.cpp:240-247) */
            const Point2 samplePos = Point2(p) + (sampler->getSampleCount() == 1 ? Vector2(0.5f)
                                                                                : Vector2(rRec.nextSample2D()));
            RayDifferential ray;
            sensor->sampleRayDifferential(ray, samplePos, Point2(0.5f), 0.5f);
            const uint32_t owner_id = (uint32_t) pos.size();
            pos.push_back(samplePos);
            Spectrum weight(1.0f), throughput(m_initialSpecularThroughput);
            for (uint32_t depth = 0; depth < 256; ++depth) {
                if (!rRec.rayIntersect(ray)) break;
                const Intersection &its = rRec.its;
                const BSDF *bsdf = its.getBSDF();
                const unsigned int type = bsdf->getType();
                alvrl_gather_rec r;
                for (int k = 0; k < 3; ++k) {
                    r.o[k] = (float) ray.o[k]; r.d[k] = (float) ray.d[k];
                    r.p[k] = (float) its.p[k]; r.n[k] = (float) its.shFrame.n[k];
                }
                const bool smooth = (type & BSDF::ESmooth) != 0;
                Spectrum rho = smooth ? bsdf->getDiffuseReflectance(its) : Spectrum(0.0f);
                put3(r.albedo, rho);
                r.flags = ALVRL_REC_HIT | (smooth ? ALVRL_REC_SMOOTH : ALVRL_REC_DELTA) |
                    (rRec.medium && !rRec.medium->getSigmaS().isZero() ? ALVRL_REC_MEDIUM : 0u);
                put3(r.weight, weight);
                r.depth = depth | ((uint32_t) j << 16);   /* the sample keys the gather's streams */
                recs.push_back(r);
                ids.push_back(pid);
                slice.push_back(sl);
                owner.push_back(owner_id);
                if (!(type & BSDF::EDelta)) break;
                /* the delta component, transmittance, roulette (:450-510) */
                MediumSamplingRecord mRec;
                Spectrum tr(1.0f);
                if (rRec.medium) {
                    rRec.medium->eval(Ray(ray, 0, its.t), mRec);
                    tr = mRec.transmittance;
                }
                if (tr.isZero()) break;
                BSDFSamplingRecord bRec(its, rRec.sampler, ERadiance);
                const Spectrum bw = bsdf->sample(bRec, Point2(0.5f));
                if (bw.isZero()) break;
                const Spectrum thr2 = throughput * tr * bw * (bRec.eta * bRec.eta);
                const Float rrProb = std::min((Float) (rRec.depth >= m_specRRdepth ? 0.98f : 1.0f), thr2.max());
                if (rrProb <= 0 || (rrProb < 1 && rRec.nextSample1D() > rrProb)) break;
                throughput = thr2 / rrProb;
                weight = weight * tr * bw / rrProb;
                RadianceQueryRecord rRec2;
                rRec2.recursiveQuery(rRec);
                ray = RayDifferential(its.p, its.toWorld(bRec.wo), ray.time);
                if (its.isMediumTransition())
                    rRec2.medium = its.getTargetMedium(ray.d);
                rRec = rRec2;
            }
            sampler->advance();
          }
        }
        const uint32_t n = (uint32_t) recs.size();
        std::vector<float> rgb((size_t) 3 * n);
        if (n) {
            if (clustered)
                checkDevice(alvrl_gather_clustered_host(ctx, &recs[0], &ids[0], &slice[0], n, &rgb[0]), ctx,
                    "alvrl_gather_clustered_host");
            else
                checkDevice(alvrl_gather_brute_host(ctx, &recs[0], &ids[0], n, &rgb[0]), ctx,
                    "alvrl_gather_brute_host");
        }
        std::vector<Spectrum> L(pos.size(), Spectrum(0.0f));
        for (uint32_t k = 0; k < n; ++k) {
            Spectrum s;
            s.fromLinearRGB(rgb[3 * k], rgb[3 * k + 1], rgb[3 * k + 2]);
            L[owner[k]] += s;
        }
        Float alpha = 1.0f;
        for (size_t i = 0; i < pos.size() && !stop; ++i)
            block->put(pos[i], L[i], alpha);   /* each sample, as renderBlock (integrator.cpp:262) */
    }

    alvrl_integrator *m_it = NULL;
    std::string m_props;   /* the integrator's properties (alvrl_integrator_create) */
    int m_sampleCount = 1;
    hipStream_t m_stream = NULL;
    int m_device = 0;
    bool m_recordsMode = false;
    float m_samplingWeight = -1.0f, m_samplingDensity = 0.0f;
    int m_strategy = ALVRL_STRATEGY_BALANCE, m_channel = 0;
    int m_specRRdepth = 100;
    Float m_initialSpecularThroughput = 20;
    alvrl_scene_desc m_desc;
    std::vector<float> m_tris;
    std::vector<uint32_t> m_mats;
    std::vector<uint32_t> m_p2s;   // records mode: the pass's slice of every pixel (column-major)
    int m_width = 0, m_height = 0;
    float *m_fb = NULL;
    /* the current pass's frame (frame mode) */
    mutable std::vector<float> m_rgb;
    mutable std::mutex m_frameLock;
    mutable std::condition_variable m_frameReady;
    mutable bool m_rendering = false;
    mutable int m_framePass = -1;
    int m_pass = 0;
};

MTS_IMPLEMENT_CLASS_S(vrlAmdIntegrator, false, ProgressiveMonteCarloIntegrator)
MTS_EXPORT_PLUGIN(vrlAmdIntegrator, "VRL integrator with Adaptive LightSlice on an MI355X (libalvrl)");
MTS_NAMESPACE_END
