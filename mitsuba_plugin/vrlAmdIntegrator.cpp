/*
 * vrlAmdIntegrator.cpp -- the vrl integrator (src/integrators/vrl/
 * vrlIntegrator.cpp) for Mitsuba 0.x with its hot path -- the per-pixel VRL
 * gather, the reduced matrix R and the per-slice cluster refinement -- on an
 * MI355X through libalvrl.so (include/alvrl.h, include/alvrl_host.h).
 *
 * Build: inside the mitsuba-ALVRL tree (src/integrators/vrl/), linked
 * against libalvrl.so and the HIP runtime, and installed as plugins/vrl.so so that scene files keep
 * type="vrl" (INTEGRATION.md "Build").  tests/test_plugin_source.py compiles
 * it here against a mock of exactly the Mitsuba declarations it uses
 * (tests/mitsuba_mock/), whose MTS_IMPLEMENT_CLASS_S expands to
 * `new vrlAmdIntegrator(stream, manager)` as class.h:219-222 does.
 *
 * Two modes, chosen by the property "amdMode":
 *
 *   "frame" (default)  The scene is described to the library once
 *                      (camera, film, the homogeneous medium's container
 *                      box and its diffuse walls, a point light, triangle
 *                      occluders with diffuse / mirror / dielectric / null
 *                      BSDFs).  The
 *                      library traces the VRLs, builds R, refines the
 *                      clusters and renders the whole frame on the GPU once
 *                      per pass; renderBlock copies its block out of that
 *                      frame.  Delta-BSDF chains are expanded by the library.
 *
 *   "records"          Mitsuba casts every eye ray itself and the library
 *                      does the per-pair work.  preprocess casts buildSlices'
 *                      ray per pixel (Preprocessor.cpp:1130-1170); prepass
 *                      casts the representative pixels' eye paths for R
 *                      (vrlIntegrator.cpp:322-330) and hands them to the
 *                      library (alvrl_integrator_prepass_records), which traces
 *                      the pass's VRLs itself (vrlTracer.h:91-230 restated,
 *                      on the GPU with gpuTracer=true) over the scene's
 *                      description -- the medium's container, the triangles
 *                      of every other shape and their BSDF classes, a point
 *                      light or an area emitter on a triangle mesh -- or
 *                      reads vrlFile, in which case any emitter and shape is
 *                      taken; it builds R and clusters; renderBlock casts the
 *                      eye paths -- LiInternal's recursion into every delta
 *                      component (:445-511) -- and gathers them in one call
 *                      per block (alvrl_gather_clustered_host).  Every
 *                      triangle of the scene (Shape::createTriMesh) is the
 *                      gathers' occluder set.  Worker threads call it
 *                      concurrently: the library gives every calling thread
 *                      its own HIP stream and scratch (alvrl.h "Threading").
 *
 * Remote workers: the integrator serializes like the reference (:210-235)
 * plus its library properties; the pass's VRLs and cluster lists travel as
 * the "vrls" and "vrlClusterInfo" resources (:353-354, 371-384) and wakeup
 * installs them (alvrl_integrator_set_vrls / _set_cluster_info).
 *
 * Properties: every property of the reference integrator, with its name and
 * default (vrlIntegrator.cpp:128-208), is parsed by the library
 * (alvrl_integrator_create).  The homogeneous medium's sampling settings are
 * private to its plugin, so the scene file repeats them on the integrator
 * when they differ from the defaults: "mediumSamplingWeight", "strategy",
 * "channel", "samplingDensity" (homogeneous.cpp:156-227).
 */
#include <mitsuba/core/plugin.h>
#include <mitsuba/core/sched.h>
#include <mitsuba/render/bsdf.h>
#include <mitsuba/render/emitter.h>
#include <mitsuba/render/medium.h>
#include <mitsuba/render/phase.h>
#include <mitsuba/render/scene.h>
#include <mitsuba/render/sensor.h>
#include <mitsuba/render/trimesh.h>

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <sstream>
#include <thread>
#include <vector>

#include "alvrl.h"
#include "alvrl_host.h"

MTS_NAMESPACE_BEGIN

namespace {

/* ALVRL_ERR_* -> Log(EError), which throws like the reference's own errors */
void check(int rc, const char *what) {
    if (rc != ALVRL_OK)
        SLog(EError, "vrl (amd): %s: %s", what, alvrl_host_last_error());
}
void checkDevice(int rc, alvrl_ctx *ctx, const char *what) {
    if (rc != ALVRL_OK)
        SLog(EError, "vrl (amd): %s: %s", what, alvrl_last_error(ctx));
}
void checkHip(hipError_t e, const char *what) {
    if (e != hipSuccess)
        SLog(EError, "vrl (amd): %s: %s", what, hipGetErrorString(e));
}

void put3(float *dst, const Spectrum &s) {
    Float r, g, b;
    s.toLinearRGB(r, g, b);
    dst[0] = (float) r; dst[1] = (float) g; dst[2] = (float) b;
}

/* The properties the library does not take (Mitsuba's own, or the medium's
 * restated on the integrator) */
bool isMitsubaOnly(const std::string &k) {
    return k == "amdMode" || k == "amdDevice" || k == "amdDevices" || k == "amdRehearseDevices" ||
        k == "mediumSamplingWeight" || k == "strategy" ||
        k == "channel" || k == "samplingDensity";
}

/* Longest eye path (records per sensor sample) the records mode follows */
const size_t kMaxPathRecords = 256;

/* "amdDevices": a comma-separated list of HIP devices ("0,1,2,3"), or
 * "all" for every visible device; empty: the one "amdDevice".  A device may
 * repeat only with the test property amdRehearseDevices=true (several
 * integrators on one GPU, exchanging through host memory) */
std::vector<int> parseDevices(const std::string &spec, int single, bool rehearse) {
    std::vector<int> out;
    if (spec.empty()) {
        out.push_back(single);
        return out;
    }
    if (spec == "all") {
        int n = 0;
        checkHip(hipGetDeviceCount(&n), "hipGetDeviceCount");
        for (int i = 0; i < n; ++i) out.push_back(i);
    } else {
        std::stringstream ss(spec);
        std::string tok;
        while (std::getline(ss, tok, ','))
            if (!tok.empty()) out.push_back(std::stoi(tok));
    }
    if (out.empty())
        SLog(EError, "vrl (amd): amdDevices lists no device");
    for (size_t i = 0; i < out.size(); ++i)
        for (size_t j = 0; j < i; ++j)
            if ((out[i] == out[j] && !rehearse) || out[i] < 0)
                SLog(EError, "vrl (amd): amdDevices must list distinct devices");
    return out;
}

} // namespace

/* The pass's VRLs as a scheduler resource ("vrls", :353): nine float planes
 * and the particle count. */
class AmdVrlSet : public SerializableObject {
public:
    AmdVrlSet() : m_particles(0), m_pass(0) { }
    AmdVrlSet(Stream *stream, InstanceManager *manager) {
        m_pass = stream->readUInt();
        m_particles = stream->readULong();
        m_soa.resize((size_t) stream->readULong());
        if (!m_soa.empty()) stream->readSingleArray(&m_soa[0], m_soa.size());
    }
    void serialize(Stream *stream, InstanceManager *manager) const {
        stream->writeUInt(m_pass);
        stream->writeULong(m_particles);
        stream->writeULong(m_soa.size());
        if (!m_soa.empty()) stream->writeSingleArray(&m_soa[0], m_soa.size());
    }
    uint32_t count() const { return (uint32_t) (m_soa.size() / 9); }
    std::vector<float> m_soa;
    uint64_t m_particles;
    uint32_t m_pass;
    MTS_DECLARE_CLASS()
};

/* The pass's cluster lists ("vrlClusterInfo", :354), in vrlClusterInfo's
 * stream layout (:66-101: m_slices, per-slice ids, per-slice weights, global
 * and fall-back lists), preceded by the pass number. */
class AmdClusterInfo : public SerializableObject {
public:
    AmdClusterInfo() : m_pass(0) { }
    AmdClusterInfo(Stream *stream, InstanceManager *manager) {
        m_pass = stream->readUInt();
        m_slices.resize((size_t) stream->readULong());
        for (size_t i = 0; i < m_slices.size(); ++i) m_slices[i] = stream->readUInt();
        const size_t ns = (size_t) stream->readULong();
        m_off.assign(ns + 1, 0);
        std::vector<std::vector<uint32_t> > ids(ns);
        for (size_t s = 0; s < ns; ++s) {
            ids[s].resize((size_t) stream->readULong());
            for (size_t k = 0; k < ids[s].size(); ++k) ids[s][k] = stream->readUInt();
            m_off[s + 1] = m_off[s] + (uint32_t) ids[s].size();
        }
        if ((size_t) stream->readULong() != ns) SLog(EError, "vrlClusterInfo: slice counts differ");
        for (size_t s = 0; s < ns; ++s) {
            if ((size_t) stream->readULong() != ids[s].size()) SLog(EError, "vrlClusterInfo: list sizes differ");
            for (size_t k = 0; k < ids[s].size(); ++k) {
                m_reps.push_back(ids[s][k]);
                m_w.push_back(stream->readFloat());
            }
        }
        for (size_t n = (size_t) stream->readULong(), i = 0; i < n; ++i) stream->readUInt();    /* global (unused, :163) */
        for (size_t n = (size_t) stream->readULong(), i = 0; i < n; ++i) stream->readFloat();
        m_fbReps.resize((size_t) stream->readULong());
        for (size_t i = 0; i < m_fbReps.size(); ++i) m_fbReps[i] = stream->readUInt();
        m_fbW.resize((size_t) stream->readULong());
        for (size_t i = 0; i < m_fbW.size(); ++i) m_fbW[i] = (float) stream->readFloat();
    }
    void serialize(Stream *stream, InstanceManager *manager) const {
        stream->writeUInt(m_pass);
        stream->writeULong(m_slices.size());
        for (size_t i = 0; i < m_slices.size(); ++i) stream->writeUInt(m_slices[i]);
        const size_t ns = m_off.empty() ? 0 : m_off.size() - 1;
        stream->writeULong(ns);
        for (size_t s = 0; s < ns; ++s) {
            stream->writeULong(m_off[s + 1] - m_off[s]);
            for (uint32_t k = m_off[s]; k < m_off[s + 1]; ++k) stream->writeUInt(m_reps[k]);
        }
        stream->writeULong(ns);
        for (size_t s = 0; s < ns; ++s) {
            stream->writeULong(m_off[s + 1] - m_off[s]);
            for (uint32_t k = m_off[s]; k < m_off[s + 1]; ++k) stream->writeFloat(m_w[k]);
        }
        stream->writeULong(0);
        stream->writeULong(0);
        stream->writeULong(m_fbReps.size());
        for (size_t i = 0; i < m_fbReps.size(); ++i) stream->writeUInt(m_fbReps[i]);
        stream->writeULong(m_fbW.size());
        for (size_t i = 0; i < m_fbW.size(); ++i) stream->writeFloat(m_fbW[i]);
    }
    std::vector<uint32_t> m_slices, m_off, m_reps, m_fbReps;
    std::vector<float> m_w, m_fbW;
    uint32_t m_pass;
    MTS_DECLARE_CLASS()
};

class vrlAmdIntegrator : public ProgressiveMonteCarloIntegrator {
public:
    vrlAmdIntegrator(const Properties &props) : ProgressiveMonteCarloIntegrator(props) {
        const std::string mode = props.getString("amdMode", "frame");
        if (mode != "frame" && mode != "records")
            Log(EError, "amdMode must be \"frame\" or \"records\"");
        m_recordsMode = mode == "records";
        m_device = props.getInteger("amdDevice", 0);
        m_rehearse = props.getBoolean("amdRehearseDevices", false);
        m_devices = parseDevices(props.getString("amdDevices", ""), m_device, m_rehearse);
        m_device = m_devices[0];
        if (m_recordsMode && m_devices.size() > 1)
            Log(EError, "vrl (amd): amdDevices (one library integrator per GPU) needs amdMode=frame");
        m_samplingWeight = props.getFloat("mediumSamplingWeight", -1);
        std::string strategy = props.getString("strategy", "balance");
        if (strategy == "balance") m_strategy = ALVRL_STRATEGY_BALANCE;
        else if (strategy == "single") m_strategy = ALVRL_STRATEGY_SINGLE;
        else if (strategy == "manual") m_strategy = ALVRL_STRATEGY_MANUAL;
        else if (strategy == "maximum") m_strategy = ALVRL_STRATEGY_MAXIMUM;
        else Log(EError, "Specified an unknown sampling strategy");
        m_channel = props.getInteger("channel", -1) + 1;
        m_samplingDensity = props.getFloat("samplingDensity", 0.0f);
        /* the reference's serialized fields (:212-218) and what records mode reads itself */
        m_volVolSamples = props.getInteger("volVolSamples", 2);
        m_volSurfSamples = props.getInteger("volSurfSamples", 2);
        m_globalCluster = props.getBoolean("globalCluster", false);
        m_localRefinement = props.getBoolean("localRefinement", true);
        m_specRRdepth = props.getInteger("specularForcedRRdepth", 100);
        m_initialSpecularThroughput = props.getFloat("initialSpecularThroughput", 20);
        m_shortVrls = props.getBoolean("shortVrls", true);
        m_vrlFile = props.getString("vrlFile", "");

        std::vector<std::string> names;
        props.putPropertyNames(names);
        std::ostringstream oss;
        for (size_t i = 0; i < names.size(); ++i) {
            if (isMitsubaOnly(names[i]))
                continue;
            oss << names[i] << "=" << props.getAsString(names[i]) << ";";
        }
        m_props = oss.str();
        create(1);
    }

    /* unserialization (vrlIntegrator.cpp:210-221): the reference's fields,
     * then this plugin's own; the library integrator is re-created from them */
    vrlAmdIntegrator(Stream *stream, InstanceManager *manager)
        : ProgressiveMonteCarloIntegrator(stream, manager) {
        m_volVolSamples = stream->readInt();
        m_volSurfSamples = stream->readInt();
        m_globalCluster = stream->readBool();
        m_localRefinement = stream->readBool();
        m_specRRdepth = stream->readInt();
        m_initialSpecularThroughput = stream->readFloat();
        m_shortVrls = stream->readBool();
        m_props = stream->readString();
        m_recordsMode = stream->readBool();
        m_device = stream->readInt();
        m_samplingWeight = (float) stream->readFloat();
        m_strategy = stream->readInt();
        m_channel = stream->readInt();
        m_samplingDensity = (float) stream->readFloat();
        m_sampleCount = stream->readInt();
        m_devices.resize((size_t) stream->readInt());
        for (size_t i = 0; i < m_devices.size(); ++i) m_devices[i] = stream->readInt();
        m_rehearse = stream->readBool();
        m_vrlsID = m_ciID = 0;
        create(m_sampleCount);
    }

    void serialize(Stream *stream, InstanceManager *manager) const {
        ProgressiveMonteCarloIntegrator::serialize(stream, manager);
        stream->writeInt(m_volVolSamples);
        stream->writeInt(m_volSurfSamples);
        stream->writeBool(m_globalCluster);
        stream->writeBool(m_localRefinement);
        stream->writeInt(m_specRRdepth);
        stream->writeFloat(m_initialSpecularThroughput);
        stream->writeBool(m_shortVrls);
        stream->writeString(m_props);
        stream->writeBool(m_recordsMode);
        stream->writeInt(m_device);
        stream->writeFloat(m_samplingWeight);
        stream->writeInt(m_strategy);
        stream->writeInt(m_channel);
        stream->writeFloat(m_samplingDensity);
        stream->writeInt(m_sampleCount);
        stream->writeInt((int) m_devices.size());
        for (size_t i = 0; i < m_devices.size(); ++i) stream->writeInt(m_devices[i]);
        stream->writeBool(m_rehearse);
    }

    ~vrlAmdIntegrator() {
        if (m_fb) hipFree(m_fb);
        if (m_stream) hipStreamDestroy(m_stream);
        if (m_it) alvrl_integrator_destroy(m_it);
        releaseMore();
        if (m_localEx) alvrl_local_exchange_destroy(m_localEx);
        if (m_devEx) alvrl_device_exchange_destroy(m_devEx);
    }

    bool preprocess(const Scene *scene, RenderQueue *queue, const RenderJob *job,
            int sceneResID, int sensorResID, int samplerResID) {
        if (!ProgressiveMonteCarloIntegrator::preprocess(scene, queue, job, sceneResID,
                sensorResID, samplerResID))
            return false;
        /* the sampler's sampleCount: sensor samples per pixel and pass
           (renderBlock's sample loop, integrator.cpp:240-264); the frame
           mode's library integrator jitters them itself */
        const Sampler *smp = static_cast<Sampler *>(Scheduler::getInstance()->getResource(samplerResID, 0));
        const size_t spp = smp->getSampleCount();
        if (spp < 1 || spp > 65535)
            Log(EError, "sampleCount must be in [1, 65535], got %d", (int) spp);
        create((int) spp);
        setUp(scene, true);
        return true;
    }

    /* vrlIntegrator::prepass (:270-356): VRLs, representatives, R, clusters */
    bool prepass(const Scene *scene, Sampler *sampler) {
        if (m_recordsMode)
            prepassRecords(scene, sampler);
        else if (m_more.empty())
            check(alvrl_integrator_prepass(m_it, m_pass), "alvrl_integrator_prepass");
        else
            prepassDevices();
        if (!m_recordsMode) {   /* the pass's slice map, for Li */
            m_p2s.clear();
            if (alvrl_integrator_num_slices(m_it)) {
                m_p2s.resize((size_t) m_width * m_height);
                check(alvrl_integrator_slices(m_it, &m_p2s[0], (uint32_t) m_p2s.size()), "alvrl_integrator_slices");
            }
        }
        publishResources();
        std::lock_guard<std::mutex> g(m_frameLock);
        m_framePass = -1;   // the frame of the new pass is rendered on first use
        ++m_pass;
        return true;
    }

    /* the pass's VRLs and cluster info as scheduler resources (:353-354) */
    void bindUsedResources(ParallelProcess *proc) const {
        ProgressiveMonteCarloIntegrator::bindUsedResources(proc);
        if (m_vrlsID) proc->bindResource("vrls", m_vrlsID);
        if (m_ciID) proc->bindResource("vrlClusterInfo", m_ciID);
    }

    /* a render worker (renderproc.cpp:52-66): install the resources it
     * received instead of running the prepass (:378-384).  Every local worker
     * of the master process calls this on the master's own instance
     * (Scheduler::getResource hands local workers the registered object), so
     * the objects this instance published itself are skipped: its prepass
     * already holds them, and installing them would pin its VRLs (set_vrls
     * is the vrlFile mode) and race the workers already in renderBlock.  A
     * remote process installs each received pass once, under a lock. */
    void wakeup(ConfigurableObject *parent, std::map<std::string, SerializableObject *> &params) {
        ProgressiveMonteCarloIntegrator::wakeup(parent, params);
        std::map<std::string, SerializableObject *>::iterator v = params.find("vrls");
        std::map<std::string, SerializableObject *>::iterator c = params.find("vrlClusterInfo");
        if (v == params.end())
            return;
        std::lock_guard<std::mutex> install(m_wakeLock);
        if (v->second == m_pubVrls)
            return;
        /* a pass is identified by its number, not by the object's address (a
           later pass's set can be allocated where the freed previous one was) */
        const int64_t passKey = (int64_t) static_cast<const AmdVrlSet *>(v->second)->m_pass
            + (c != params.end() ? ((int64_t) static_cast<const AmdClusterInfo *>(c->second)->m_pass + 1) << 32 : 0);
        if (passKey == m_installedPass)
            return;
        const Scene *scene = static_cast<const Scene *>(parent);
        if (!m_ready && scene)
            setUp(scene, false);
        const AmdVrlSet *vs = static_cast<const AmdVrlSet *>(v->second);
        for (size_t k = 0; k <= m_more.size(); ++k) {   /* every device's integrator */
            alvrl_integrator *it = k ? m_more[k - 1] : m_it;
            check(alvrl_integrator_set_vrls(it, vs->count() ? &vs->m_soa[0] : NULL, vs->count(),
                                            std::max<uint64_t>(vs->m_particles, 1)), "alvrl_integrator_set_vrls");
            if (c != params.end()) {
                const AmdClusterInfo *ci = static_cast<const AmdClusterInfo *>(c->second);
                check(alvrl_integrator_set_cluster_info(it, ci->m_pass, (uint32_t) ci->m_slices.size(),
                          ci->m_slices.empty() ? NULL : &ci->m_slices[0], (uint32_t) ci->m_off.size() - 1,
                          &ci->m_off[0], ci->m_reps.empty() ? NULL : &ci->m_reps[0], ci->m_w.empty() ? NULL : &ci->m_w[0],
                          (uint32_t) ci->m_fbReps.size(), ci->m_fbReps.empty() ? NULL : &ci->m_fbReps[0],
                          ci->m_fbW.empty() ? NULL : &ci->m_fbW[0]), "alvrl_integrator_set_cluster_info");
                m_p2s = ci->m_slices;
                m_pass = (int) ci->m_pass;
            } else {
                check(alvrl_integrator_prepass(it, vs->m_pass), "alvrl_integrator_prepass");   /* brute force */
                m_pass = (int) vs->m_pass;
            }
        }
        m_installedPass = passKey;
        std::lock_guard<std::mutex> g(m_frameLock);
        m_framePass = -1;
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

    /* Li (vrlIntegrator.cpp:386-393) for a caller outside renderBlock:
     * LiInternal's eye path of 'ray' as gather records (appendPath, both
     * modes cast it with Mitsuba's scene), the slice of the image position
     * the sensor gives the ray (getSamplePosition, :551-560; m_slices[y +
     * H*x]) and one gather over the pass's clusters, or over every VRL
     * without clustering (getVRLContributions, :792-825).  The pixel keys the
     * gathers' counter streams as in renderBlock. */
    Spectrum Li(const RayDifferential &ray, RadianceQueryRecord &rRec) const {
        std::vector<alvrl_gather_rec> recs;
        /* the sampler's sample index keys this call's counter streams (depth
           word, sampleIndex << 16), so repeated calls for one pixel draw
           fresh uniforms as the reference's rRec.sampler does */
        const uint32_t sampleIndex = rRec.sampler ? (uint32_t) (rRec.sampler->getSampleIndex() & 0xFFFFu) : 0u;
        appendPath(ray, rRec, Spectrum(1.0f), Spectrum(m_initialSpecularThroughput), sampleIndex, &recs);
        const uint32_t n = (uint32_t) recs.size();
        if (!n)
            return Spectrum(0.0f);
        PositionSamplingRecord pRec;
        pRec.p = ray.o;
        DirectionSamplingRecord dRec(ray.d);
        Point2 pos;
        rRec.scene->getSensor()->getSamplePosition(pRec, dRec, pos);
        const int x = std::min(std::max((int) pos.x, 0), m_width - 1);
        const int y = std::min(std::max((int) pos.y, 0), m_height - 1);
        const std::vector<uint32_t> ids(n, (uint32_t) y * (uint32_t) m_width + (uint32_t) x);
        std::vector<float> rgb((size_t) 3 * n);
        alvrl_ctx *ctx = alvrl_integrator_ctx(m_it);
        if (!m_p2s.empty()) {
            const std::vector<uint32_t> slice(n, m_p2s[(size_t) y + (size_t) m_height * x]);
            checkDevice(alvrl_gather_clustered_host(ctx, &recs[0], &ids[0], &slice[0], n, &rgb[0]), ctx,
                "alvrl_gather_clustered_host (Li)");
        } else {
            checkDevice(alvrl_gather_brute_host(ctx, &recs[0], &ids[0], n, &rgb[0]), ctx,
                "alvrl_gather_brute_host (Li)");
        }
        Spectrum L(0.0f);
        for (uint32_t k = 0; k < n; ++k) {
            Spectrum s;
            s.fromLinearRGB(rgb[3 * k], rgb[3 * k + 1], rgb[3 * k + 2]);
            L += s;
        }
        return L;
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
    /* the library integrator for 'spp' sensor samples per pixel */
    void create(int spp) {
        if (m_it && spp == m_sampleCount)
            return;
        if (m_it) alvrl_integrator_destroy(m_it);
        m_it = NULL;
        m_sampleCount = spp;
        releaseMore();
        std::ostringstream oss;
        oss << m_props << "sampleCount=" << spp << ";";
        check(alvrl_integrator_create(oss.str().c_str(), m_device, &m_it), "alvrl_integrator_create");
        if (!m_stream) {
            checkHip(hipSetDevice(m_device), "hipSetDevice");
            checkHip(hipStreamCreateWithFlags(&m_stream, hipStreamNonBlocking), "hipStreamCreate");
        }
        /* amdDevices: one more library integrator per further GPU, the same
           properties (and so the same VRLs, slices and streams) */
        for (size_t k = 1; k < m_devices.size(); ++k) {
            alvrl_integrator *it = NULL;
            check(alvrl_integrator_create(oss.str().c_str(), m_devices[k], &it), "alvrl_integrator_create");
            m_more.push_back(it);
            hipStream_t st = NULL;
            checkHip(hipSetDevice(m_devices[k]), "hipSetDevice");
            checkHip(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
            m_moreStreams.push_back(st);
        }
        ensureExchange();
        m_ready = false;
    }

    /* the scene to the library: the descriptor (frame mode) or, in records
     * mode, buildSlices' gather points (only on the master: 'slicing') */
    void setUp(const Scene *scene, bool slicing) {
        const Vector2i size = scene->getSensor()->getFilm()->getSize();
        const Vector2i crop = scene->getSensor()->getFilm()->getCropSize();
        if (size.x != crop.x || size.y != crop.y)
            Log(EError, "vrl (amd): crop windows are not supported (m_slices covers the whole film)");
        m_width = size.x; m_height = size.y;
        if (m_recordsMode) {
            describeExt(scene, slicing);
        } else {
            describe(scene);
            alvrl_scene_desc sd = m_desc;
            bindDesc(&sd, m_tris, m_mats, m_emit, m_albs);
            check(alvrl_integrator_preprocess(m_it, &sd), "alvrl_integrator_preprocess");
            for (size_t k = 0; k < m_more.size(); ++k)
                check(alvrl_integrator_preprocess(m_more[k], &sd), "alvrl_integrator_preprocess");
        }
        m_rgb.assign((size_t) 3 * m_width * m_height, 0.0f);
        if (m_fb) hipFree(m_fb);
        m_fb = NULL;
        if (!m_recordsMode) {
            checkHip(hipSetDevice(m_device), "hipSetDevice");
            checkHip(hipMalloc(&m_fb, sizeof(float) * m_rgb.size()), "hipMalloc");
        }
        for (size_t k = 0; k < m_moreFb.size(); ++k) {
            checkHip(hipSetDevice(m_devices[k + 1]), "hipSetDevice");
            checkHip(hipFree(m_moreFb[k]), "hipFree");
        }
        m_moreFb.assign(m_more.size(), (float *) NULL);
        m_moreRgb.assign(m_more.size(), std::vector<float>());
        for (size_t k = 0; k < m_more.size(); ++k) {
            checkHip(hipSetDevice(m_devices[k + 1]), "hipSetDevice");
            checkHip(hipMalloc(&m_moreFb[k], sizeof(float) * m_rgb.size()), "hipMalloc");
            m_moreRgb[k].assign(m_rgb.size(), 0.0f);
        }
        m_ready = true;
    }

    /* the one homogeneous medium, in the library's terms */
    const Medium *describeMedium(const Scene *scene, alvrl_medium_desc *md) const {
        const Medium *medium = scene->getSensor()->getMedium();
        if (scene->getMedia().size() != 1)
            Log(EError, "vrl (amd) needs exactly one (homogeneous) medium, the one the VRLs live in");
        if (!medium) medium = scene->getMedia()[0].get();
        if (medium->getClass()->getName() != "HomogeneousMedium")
            Log(EError, "vrl (amd): the medium must be homogeneous");
        const Spectrum ss = medium->getSigmaS(), sa = medium->getSigmaA();
        for (int i = 0; i < 3; ++i) {
            md->sigma_s[i] = (float) ss[i];
            md->sigma_a[i] = (float) sa[i];
        }
        md->sampling_weight = m_samplingWeight;
        md->strategy = m_strategy;
        md->channel = m_channel;
        md->sampling_density = m_samplingDensity;
        const PhaseFunction *phase = medium->getPhaseFunction();
        const std::string pn = phase->getClass()->getName();
        if (pn != "HGPhaseFunction" && pn != "IsotropicPhaseFunction")
            Log(EError, "vrl (amd): the phase function must be isotropic or hg");
        const bool hg = pn == "HGPhaseFunction";
        md->phase_type = hg ? 1 : 0;
        md->phase_g = hg ? (float) phase->getMeanCosine() : 0.0f;
        return medium;
    }

    /* The scene in the library's terms (alvrl_scene_desc), frame mode: the
     * perspective camera, then the light transport (describeTransport) */
    void describe(const Scene *scene) {
        alvrl_scene_default(&m_desc, 1, 1);
        const Sensor *sensor = scene->getSensor();
        const PerspectiveCamera *cam = dynamic_cast<const PerspectiveCamera *>(sensor);
        if (!cam)
            Log(EError, "vrl (amd) frame mode needs a perspective camera (amdMode=records takes any sensor)");
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
        m_desc.width = m_width; m_desc.height = m_height;
        if (!sensor->getMedium())
            Log(EError, "vrl (amd) frame mode needs the camera inside the medium (amdMode=records does not)");
        describeTransport(scene, false, &m_desc, &m_tris, &m_mats, &m_emit, &m_albs);
    }

    /* The light transport the library's VRL tracer (and, in frame mode, its
     * eye rays) sees: the medium and the shape that contains it, the one
     * emitter -- a point light or an area emitter on a triangle mesh -- and
     * every other shape's triangles with its BSDF class.  Frame mode renders
     * from it; records mode traces the pass's VRLs over it
     * (alvrl_scene_ext::tracer) and refuses a scene it cannot express unless
     * a vrlFile supplies the VRLs. */
    void describeTransport(const Scene *scene, bool records, alvrl_scene_desc *d, std::vector<float> *tris,
            std::vector<uint32_t> *mats, std::vector<float> *emit, std::vector<float> *albs) {
        const char *alt = records ? "records mode traces the VRLs over the scene's description; "
                                    "a vrlFile takes any scene" : "amdMode=records takes any";
        const char *mode = records ? "records" : "frame";
        const Medium *medium = describeMedium(scene, &d->medium);

        /* the one emitter: a point light (samplePosition returns its power,
           intensity * 4 pi, point.cpp:81-91) or an area emitter on a triangle
           mesh (alvrl_scene_desc::emitter_tris; its radiance from
           evalPosition = radiance * pi, area.cpp:100-102) */
        if (scene->getEmitters().size() != 1)
            Log(EError, "vrl (amd) %s mode needs exactly one emitter (%s)", mode, alt);
        const Emitter *light = scene->getEmitters()[0].get();
        PositionSamplingRecord pRec(0.0f);
        const Spectrum power = light->samplePosition(pRec, Point2(0.5f));
        emit->clear();
        if (light->getType() & Emitter::EDeltaPosition) {
            put3(d->light_intensity, power * (Float) (0.25f * INV_PI));
            for (int i = 0; i < 3; ++i) d->light_pos[i] = (float) pRec.p[i];
        } else if (light->getType() & Emitter::EOnSurface) {
            const TriMesh *lmesh = NULL;
            for (size_t s = 0; s < scene->getShapes().size(); ++s)
                if (scene->getShapes()[s]->isEmitter() && scene->getShapes()[s]->getEmitter() == light)
                    lmesh = dynamic_cast<const TriMesh *>(scene->getShapes()[s].get());
            if (!lmesh)
                Log(EError, "vrl (amd) %s mode: the area emitter must sit on a triangle mesh (%s)", mode, alt);
            appendEmitterTriangles(lmesh, emit);
            put3(d->emitter_radiance, light->evalPosition(pRec) * (Float) INV_PI);
        } else {
            Log(EError, "vrl (amd) %s mode needs a point light or an area emitter (%s)", mode, alt);
        }

        /* the container: the shape whose interior is the medium; its walls' diffuse reflectance.
           Every other shape's triangles carry their own diffuse reflectance
           (occluder_albedos): an emitter's mesh, to which Mitsuba gives an
           all-absorbing SmoothDiffuse (shape.cpp:49-56), absorbs */
        tris->clear(); mats->clear(); albs->clear();
        bool haveBox = false, haveSpec = false, haveEta = false;
        const ref_vector<Shape> &shapes = scene->getShapes();
        for (size_t s = 0; s < shapes.size(); ++s) {
            const Shape *sh = shapes[s].get();
            const BSDF *bsdf = sh->getBSDF();
            Intersection its;
            if (sh->getInteriorMedium() == medium && !haveBox) {
                const AABB box = sh->getAABB();
                for (int i = 0; i < 3; ++i) {
                    d->box_min[i] = (float) box.min[i];
                    d->box_max[i] = (float) box.max[i];
                }
                if (bsdf) put3(d->albedo, diffuseReflectance(sh, bsdf, mode, alt, true));
                haveBox = true;
                /* a container that is not the box itself (a rotated or curved
                   mesh) bounds the medium with its own triangles; on the box's
                   faces they tie with its walls, which win */
                if (const TriMesh *cm = dynamic_cast<const TriMesh *>(sh)) {
                    if (!onBoxFaces(cm, box)) {
                        const Spectrum rho = diffuseReflectance(sh, bsdf, mode, alt, false);
                        appendTriangles(cm, ALVRL_MAT_DIFFUSE, tris, mats);
                        appendAlbedo(rho, mats->size(), albs);
                    }
                }
                continue;
            }
            const TriMesh *mesh = dynamic_cast<const TriMesh *>(sh);
            if (!mesh)
                Log(EError, "vrl (amd) %s mode: shape \"%s\" inside the medium is not a triangle mesh (%s)",
                    mode, sh->getName().c_str(), alt);
            uint32_t mat = ALVRL_MAT_DIFFUSE;
            Spectrum rho(0.0f);   /* the diffuse reflectance (delta and null BSDFs: unused) */
            if (bsdf) {
                const unsigned int type = bsdf->getType();
                if (type & BSDF::ENull) {
                    mat = ALVRL_MAT_NULL;
                } else if ((type & BSDF::EDeltaReflection) && !(type & BSDF::EDeltaTransmission) &&
                           !(type & BSDF::ESmooth)) {
                    mat = ALVRL_MAT_MIRROR;
                    if (!haveSpec) put3(d->occluder_specular, bsdf->getSpecularReflectance(its));
                    haveSpec = true;
                } else if ((type & BSDF::EDeltaReflection) && (type & BSDF::EDeltaTransmission) &&
                           !(type & BSDF::ESmooth)) {
                    /* smooth dielectric (dielectric.cpp): both delta components */
                    mat = ALVRL_MAT_DIELECTRIC;
                    if (haveEta && (float) bsdf->getEta() != d->occluder_eta)
                        Log(EError, "vrl (amd) %s mode: dielectrics with different IORs (%s)", mode, alt);
                    d->occluder_eta = (float) bsdf->getEta();
                    haveEta = true;
                } else if (type & BSDF::EDelta) {
                    Log(EError, "vrl (amd) %s mode: BSDF of \"%s\" is neither diffuse, mirror, dielectric nor "
                        "null (%s)", mode, sh->getName().c_str(), alt);
                } else {
                    rho = diffuseReflectance(sh, bsdf, mode, alt);
                }
            }
            appendTriangles(mesh, mat, tris, mats);
            appendAlbedo(rho, mats->size(), albs);
        }
        if (!haveBox)
            Log(EError, "vrl (amd) needs a shape that contains the medium (its interior)");
        bindDesc(d, *tris, *mats, *emit, *albs);
    }

    /* the reflectance of the triangles appended last, up to n triangles in all */
    static void appendAlbedo(const Spectrum &rho, size_t n, std::vector<float> *albs) {
        float c[3];
        put3(c, rho);
        while (albs->size() < 3 * n)
            albs->insert(albs->end(), c, c + 3);
    }

    /* point a descriptor at the arrays that hold its triangles */
    static void bindDesc(alvrl_scene_desc *d, const std::vector<float> &tris, const std::vector<uint32_t> &mats,
            const std::vector<float> &emit, const std::vector<float> &albs) {
        d->occluders = tris.empty() ? NULL : &tris[0];
        d->occluder_material = mats.empty() ? NULL : &mats[0];
        d->n_occluders = (uint32_t) mats.size();
        d->occluder_albedos = albs.empty() ? NULL : &albs[0];
        d->emitter_tris = emit.empty() ? NULL : &emit[0];
        d->n_emitter_tris = (uint32_t) (emit.size() / 9);
    }

    /* The constant diffuse reflectance of a shape's smooth diffuse BSDF,
     * evaluated at real points of the shape (Shape::samplePosition: position,
     * normal and uv): the descriptor holds one albedo per class of surface,
     * so another smooth BSDF (its vol->surf term is not rho / pi cos) or a
     * textured reflectance is refused with a pointer to records mode */
    Spectrum diffuseReflectance(const Shape *sh, const BSDF *bsdf, const char *mode, const char *alt,
            bool container = false) const {
        /* the box's walls face the medium whatever the mesh's winding, so a
           two-sided diffuse container is the same surface */
        const std::string cls = bsdf->getClass()->getName();
        if (cls != "SmoothDiffuse" && !(container && cls == "TwoSidedBRDF"))
            Log(EError, "vrl (amd) %s mode: the BSDF of \"%s\" is %s; its walls and occluders take the "
                "smooth diffuse BSDF the gathers evaluate (diffuse.cpp:110-118; %s)", mode, sh->getName().c_str(),
                bsdf->getClass()->getName().c_str(), alt);
        const Point2 at[3] = { Point2(0.25f, 0.25f), Point2(0.5f, 0.75f), Point2(0.875f, 0.125f) };
        Spectrum first(0.0f);
        for (int k = 0; k < 3; ++k) {
            PositionSamplingRecord pRec(0.0f);
            sh->samplePosition(pRec, at[k]);
            Intersection its;
            its.t = 0.0f;
            its.p = pRec.p;
            its.uv = pRec.uv;
            its.shape = sh;
            its.geoFrame.n = pRec.n;
            its.shFrame.n = pRec.n;
            const Spectrum rho = bsdf->getDiffuseReflectance(its);
            if (k == 0)
                first = rho;
            else if (rho != first)
                Log(EError, "vrl (amd) %s mode: \"%s\" has a textured reflectance (%s)", mode,
                    sh->getName().c_str(), alt);
        }
        return first;
    }

    static void appendTriangles(const TriMesh *mesh, uint32_t mat, std::vector<float> *tris,
            std::vector<uint32_t> *mats) {
        appendTriangles(mesh, tris);
        mats->resize(tris->size() / 9, mat);
    }

    static void appendTriangles(const TriMesh *mesh, std::vector<float> *out) {
        const Point *pos = mesh->getVertexPositions();
        const Triangle *tri = mesh->getTriangles();
        for (size_t f = 0; f < mesh->getTriangleCount(); ++f)
            for (int k = 0; k < 3; ++k) {
                const Point &p = pos[tri[f].idx[k]];
                out->push_back((float) p.x);
                out->push_back((float) p.y);
                out->push_back((float) p.z);
            }
    }

    /* An area emitter's triangles for the library, which emits on the side of
     * cross(p1 - p0, p2 - p0).  Mitsuba emits on the side of the shading
     * normal Triangle::sample interpolates from the vertex normals
     * (triangle.cpp:34-42), and flipNormals negates those normals without
     * touching the winding (trimesh.cpp:623-627, 660-664; the winding is
     * swapped only without normals, :615-620): a triangle whose vertex
     * normals point against its winding normal is handed over with p0 and p1
     * swapped.  Normals that are not one direction per triangle (a curved
     * light) have no equivalent here and are refused. */
    static void appendEmitterTriangles(const TriMesh *mesh, std::vector<float> *out) {
        const Point *pos = mesh->getVertexPositions();
        const Triangle *tri = mesh->getTriangles();
        const Normal *nrm = mesh->hasVertexNormals() ? mesh->getVertexNormals() : NULL;
        for (size_t f = 0; f < mesh->getTriangleCount(); ++f) {
            int order[3] = {0, 1, 2};
            if (nrm) {
                const Point &p0 = pos[tri[f].idx[0]], &p1 = pos[tri[f].idx[1]], &p2 = pos[tri[f].idx[2]];
                const Vector g = cross(p1 - p0, p2 - p0);
                const Vector n0(nrm[tri[f].idx[0]]), n1(nrm[tri[f].idx[1]]), n2(nrm[tri[f].idx[2]]);
                const Float tol = 1e-4f;
                if (dot(n0, n1) < 1 - tol || dot(n0, n2) < 1 - tol)
                    Log(EError, "vrl (amd) frame mode: area emitter \"%s\" has smooth vertex normals (a curved "
                        "light); use faceNormals=true or amdMode=records", mesh->getName().c_str());
                if (dot(n0 + n1 + n2, g) < 0)
                    std::swap(order[0], order[1]);
            }
            for (int k = 0; k < 3; ++k) {
                const Point &p = pos[tri[f].idx[order[k]]];
                out->push_back((float) p.x);
                out->push_back((float) p.y);
                out->push_back((float) p.z);
            }
        }
    }

    /* every vertex on a face of the box: the mesh is the box itself */
    static bool onBoxFaces(const TriMesh *mesh, const AABB &box) {
        const Point *pos = mesh->getVertexPositions();
        const Triangle *tri = mesh->getTriangles();
        for (size_t f = 0; f < mesh->getTriangleCount(); ++f) {
            bool face = false;   /* all three vertices on one common face */
            for (int a = 0; a < 3 && !face; ++a)
                for (int side = 0; side < 2 && !face; ++side) {
                    const Float c = side ? box.max[a] : box.min[a];
                    face = pos[tri[f].idx[0]][a] == c && pos[tri[f].idx[1]][a] == c && pos[tri[f].idx[2]][a] == c;
                }
            if (!face)
                return false;
        }
        return true;
    }

    /* records mode: the medium, every shape's triangles for the gathers'
     * occluder test, and (on the master) buildSlices' gather point of every
     * pixel (Preprocessor.cpp:1140-1170): the centre ray's first hit,
     * continued past null surfaces */
    void describeExt(const Scene *scene, bool slicing) {
        alvrl_scene_ext e;
        std::memset(&e, 0, sizeof(e));
        e.width = m_width; e.height = m_height;
        const AABB &aabb = scene->getAABB();
        for (int i = 0; i < 3; ++i) { e.scene_min[i] = (float) aabb.min[i]; e.scene_max[i] = (float) aabb.max[i]; }
        m_medium = describeMedium(scene, &e.medium);
        m_tris.clear(); m_mats.clear();
        const ref_vector<Shape> &shapes = scene->getShapes();
        for (size_t s = 0; s < shapes.size(); ++s) {
            Shape *sh = const_cast<Shape *>(shapes[s].get());
            ref<TriMesh> mesh = sh->createTriMesh();
            if (!mesh)
                Log(EError, "vrl (amd): shape \"%s\" has no triangle mesh for the gathers' visibility",
                    sh->getName().c_str());
            const BSDF *bsdf = sh->getBSDF();
            uint32_t mat = ALVRL_MAT_DIFFUSE;
            if (bsdf && (bsdf->getType() & BSDF::ENull)) mat = ALVRL_MAT_NULL;
            else if (bsdf && (bsdf->getType() & BSDF::EDeltaTransmission)) mat = ALVRL_MAT_DIELECTRIC;
            else if (bsdf && (bsdf->getType() & BSDF::EDelta)) mat = ALVRL_MAT_MIRROR;
            appendTriangles(mesh.get(), mat, &m_tris, &m_mats);
        }
        e.triangles = m_tris.empty() ? NULL : &m_tris[0];
        e.n_triangles = (uint32_t) m_mats.size();
        e.triangle_material = m_mats.empty() ? NULL : &m_mats[0];
        std::vector<alvrl_gather_rec> sl;
        if (slicing) {
            sl.resize((size_t) m_width * m_height);
            std::memset(&sl[0], 0, sizeof(alvrl_gather_rec) * sl.size());
            const Sensor *sensor = scene->getSensor();
            for (int x = 0; x < m_width; ++x) {
                for (int y = 0; y < m_height; ++y) {
                    Ray ray;
                    Intersection its;
                    sensor->sampleRay(ray, Point2(x + 0.5f, y + 0.5f), Point2(0.0f), 0.0f);
                    if (!scene->rayIntersect(ray, its))
                        continue;   /* no gather point: no slice */
                    Point gp;
                    Vector n;
                    while (true) {
                        gp = its.p;
                        n = its.shFrame.n;
                        if (!(its.getBSDF()->getType() & BSDF::ENull))
                            break;
                        ray = Ray(ray, its.t + Epsilon, ray.maxt);
                        if (!scene->rayIntersect(ray, its))
                            break;
                    }
                    alvrl_gather_rec &r = sl[(size_t) y * m_width + x];
                    for (int k = 0; k < 3; ++k) { r.p[k] = (float) gp[k]; r.n[k] = (float) n[k]; }
                    r.flags = ALVRL_REC_HIT;
                }
            }
        }
        e.slice_recs = sl.empty() ? NULL : &sl[0];
        /* the VRL tracer's view of the scene (vrlTracer.h:91-230 runs in the
           library, every pass): needed unless a vrlFile supplies the VRLs */
        if (m_vrlFile.empty()) {
            alvrl_scene_default(&m_tdesc, 1, 1);
            describeTransport(scene, true, &m_tdesc, &m_ttris, &m_tmats, &m_temit, &m_talbs);
            e.tracer = &m_tdesc;
        }
        check(alvrl_integrator_preprocess_ext(m_it, &e), "alvrl_integrator_preprocess_ext");
    }

    /* records mode prepass: the library traces the pass's VRLs over the
     * scene's description (alvrl_scene_ext::tracer, vrl tracing :276-280) or
     * has read vrlFile in preprocess (:243-252); then R over the host's eye
     * paths */
    void prepassRecords(const Scene *scene, Sampler *sampler) {
        if (!m_globalCluster && !m_localRefinement) {
            check(alvrl_integrator_prepass(m_it, m_pass), "alvrl_integrator_prepass");   /* brute force */
            m_p2s.clear();
            return;
        }
        uint32_t nrows = 0;
        check(alvrl_integrator_rep_pixels(m_it, m_pass, NULL, 0, &nrows), "alvrl_integrator_rep_pixels");
        std::vector<uint32_t> pix(nrows + 1);
        check(alvrl_integrator_rep_pixels(m_it, m_pass, &pix[0], nrows + 1, &nrows), "alvrl_integrator_rep_pixels");
        /* R rows (:322-330): the ray through the representative pixel's centre,
           LiInternal's eye path (getLiLuminanceVrlContributions, :527-539) */
        std::vector<alvrl_gather_rec> recs;
        std::vector<uint32_t> rows;
        const Sensor *sensor = scene->getSensor();
        for (uint32_t i = 0; i < nrows; ++i) {
            const Point2i p((int) (pix[i] % (uint32_t) m_width), (int) (pix[i] / (uint32_t) m_width));
            sampler->generate(p);
            RadianceQueryRecord rRec(scene, sampler);
            rRec.newQuery(RadianceQueryRecord::ESensorRay, sensor->getMedium());
            Ray ray0;
            sensor->sampleRay(ray0, Point2(p) + Vector2(0.5f), Point2(0.0f), 0.0f);
            const RayDifferential ray(ray0);
            appendPath(ray, rRec, Spectrum(1.0f), Spectrum(m_initialSpecularThroughput), 0u, &recs);
            rows.resize(recs.size(), i);
            sampler->advance();
        }
        check(alvrl_integrator_prepass_records(m_it, m_pass, recs.empty() ? NULL : &recs[0],
                                               rows.empty() ? NULL : &rows[0], (uint32_t) recs.size(), 0, 1, NULL),
              "alvrl_integrator_prepass_records");
        m_p2s.resize((size_t) m_width * m_height);
        check(alvrl_integrator_slices(m_it, &m_p2s[0], (uint32_t) m_p2s.size()), "alvrl_integrator_slices");
    }

    /* the pass's VRLs and cluster lists for remote workers (:353-354) */
    void publishResources() {
        ref<Scheduler> sched = Scheduler::getInstance();
        if (m_vrlsID) sched->unregisterResource(m_vrlsID);
        if (m_ciID) sched->unregisterResource(m_ciID);
        m_vrlsID = m_ciID = 0;
        ref<AmdVrlSet> vs = new AmdVrlSet();
        uint32_t n = 0;
        uint64_t pc = 0;
        check(alvrl_integrator_vrls(m_it, NULL, 0, &n, &pc), "alvrl_integrator_vrls");
        vs->m_soa.resize((size_t) 9 * n);
        if (n) check(alvrl_integrator_vrls(m_it, &vs->m_soa[0], n, &n, &pc), "alvrl_integrator_vrls");
        vs->m_particles = pc;
        vs->m_pass = (uint32_t) m_pass;
        m_vrlsID = sched->registerResource(vs);
        m_pubVrls = vs.get();
        const uint32_t ns = alvrl_integrator_num_slices(m_it);
        if (!ns)
            return;
        ref<AmdClusterInfo> ci = new AmdClusterInfo();
        ci->m_pass = (uint32_t) m_pass;
        ci->m_slices.resize((size_t) m_width * m_height);
        check(alvrl_integrator_slices(m_it, &ci->m_slices[0], (uint32_t) ci->m_slices.size()), "alvrl_integrator_slices");
        alvrl_integrator_stats st;
        check(alvrl_integrator_get_stats(m_it, &st), "alvrl_integrator_get_stats");
        ci->m_off.resize(ns + 1);
        ci->m_reps.resize((size_t) st.clusters_total + 1);
        ci->m_w.resize((size_t) st.clusters_total + 1);
        ci->m_fbReps.resize((size_t) n + 1);
        ci->m_fbW.resize((size_t) n + 1);
        uint32_t nfb = 0;
        check(alvrl_integrator_clusters(m_it, &ci->m_off[0], &ci->m_reps[0], &ci->m_w[0],
                                        (uint32_t) ci->m_reps.size(), &ci->m_fbReps[0], &ci->m_fbW[0],
                                        (uint32_t) ci->m_fbReps.size(), &nfb), "alvrl_integrator_clusters");
        ci->m_reps.resize(ci->m_off[ns]);
        ci->m_w.resize(ci->m_off[ns]);
        ci->m_fbReps.resize(nfb);
        ci->m_fbW.resize(nfb);
        m_ciID = sched->registerResource(ci);
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
        hipError_t e = hipSuccess;
        if (m_more.empty()) {
            e = renderTiles(m_it, m_device, 0, 1, m_fb, m_stream, &m_rgb[0], m_rgb.size(), &rc);
        } else {
            /* every GPU renders its 64x64 tiles (alvrl_integrator_render with
               rank k of N) on its own host thread; the tiles partition the
               frame, so the framebuffer reduce is the sum of the N frames:
               one ncclReduce into device 0's framebuffer and one copy to the
               host, or, rehearsing on one GPU, N copies summed on the host */
            const uint32_t n = (uint32_t) m_devices.size();
            std::vector<int> rcs(n, ALVRL_OK);
            std::vector<hipError_t> es(n, hipSuccess);
            std::vector<std::thread> th;
            for (uint32_t k = 0; k < n; ++k)
                th.push_back(std::thread([&, k]() {
                    float *fb = k ? m_moreFb[k - 1] : m_fb;
                    hipStream_t st = k ? m_moreStreams[k - 1] : m_stream;
                    if (m_devEx) {
                        es[k] = renderTiles(k ? m_more[k - 1] : m_it, m_devices[k], k, n, fb, st, NULL, m_rgb.size(),
                                            &rcs[k]);
                        /* every rank joins the reduce, even after a failure of
                           its own, so that no peer is left waiting in it */
                        const int rr = alvrl_device_exchange_reduce_frame(m_devEx, k, fb, m_rgb.size(), st);
                        if (rcs[k] == ALVRL_OK) rcs[k] = rr;
                        if (es[k] == hipSuccess && rcs[k] == ALVRL_OK && k == 0)
                            es[k] = hipMemcpyAsync(&m_rgb[0], fb, sizeof(float) * m_rgb.size(),
                                                   hipMemcpyDeviceToHost, st);
                        if (es[k] == hipSuccess) es[k] = hipStreamSynchronize(st);
                    } else {
                        es[k] = renderTiles(k ? m_more[k - 1] : m_it, m_devices[k], k, n, fb, st,
                                            k ? &m_moreRgb[k - 1][0] : &m_rgb[0], m_rgb.size(), &rcs[k]);
                    }
                }));
            for (size_t k = 0; k < th.size(); ++k) th[k].join();
            for (uint32_t k = 0; k < n; ++k) {
                if (e == hipSuccess) e = es[k];
                if (rc == ALVRL_OK) rc = rcs[k];
            }
            if (e == hipSuccess && rc == ALVRL_OK && !m_devEx)
                for (size_t k = 0; k < m_moreRgb.size(); ++k)
                    for (size_t i = 0; i < m_rgb.size(); ++i) m_rgb[i] += m_moreRgb[k][i];
        }
        g.lock();
        m_rendering = false;
        if (e == hipSuccess && rc == ALVRL_OK) m_framePass = m_pass;
        m_frameReady.notify_all();
        g.unlock();
        checkHip(e, "frame render");
        check(rc, "alvrl_integrator_render");
    }

    /* one device's share of the frame: zero, render rank k's tiles, copy back
       (host == NULL: leave it on the device) */
    static hipError_t renderTiles(alvrl_integrator *it, int device, uint32_t rank, uint32_t world, float *fb,
            hipStream_t st, float *host, size_t n, int *rc) {
        *rc = ALVRL_OK;
        hipError_t e = hipSetDevice(device);
        if (e == hipSuccess) e = hipMemsetAsync(fb, 0, sizeof(float) * n, st);
        if (e == hipSuccess) *rc = alvrl_integrator_render(it, rank, world, fb, st);
        if (e == hipSuccess && *rc == ALVRL_OK && host)
            e = hipMemcpyAsync(host, fb, sizeof(float) * n, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess && *rc == ALVRL_OK) e = hipStreamSynchronize(st);
        return e;
    }

    /* amdDevices: the slice-sharded prepass (alvrl_integrator_prepass_dist)
     * with one host thread per GPU and the in-process exchange: rank k
     * builds R for and refines the slices s % N == k, the non-zero mask is
     * OR-ed and the cluster lists all-gathered, so every integrator ends the
     * pass with every slice's list */
    void prepassDevices() {
        ensureExchange();
        const uint32_t n = (uint32_t) m_devices.size();
        std::vector<int> rcs(n, ALVRL_OK);
        std::vector<std::thread> th;
        for (uint32_t k = 0; k < n; ++k)
            th.push_back(std::thread([&, k]() {
                if (hipSetDevice(m_devices[k]) != hipSuccess) rcs[k] = ALVRL_ERR_HIP;
                else
                    rcs[k] = alvrl_integrator_prepass_dist(k ? m_more[k - 1] : m_it, (uint32_t) m_pass, k, n,
                                                           m_devEx ? alvrl_device_exchange_rank(m_devEx, k)
                                                                   : alvrl_local_exchange_rank(m_localEx, k));
                /* a rank that fails wakes the others at once instead of
                   leaving them in the collective it will not join */
                if (rcs[k] != ALVRL_OK) {
                    if (m_devEx) alvrl_device_exchange_abort(m_devEx);
                    else alvrl_local_exchange_abort(m_localEx);
                }
            }));
        for (size_t k = 0; k < th.size(); ++k) th[k].join();
        bool failed = false;
        for (uint32_t k = 0; k < n; ++k) failed |= rcs[k] != ALVRL_OK;
        if (failed) {   /* an aborted group is not reused: the next pass makes a new one */
            if (m_devEx) alvrl_device_exchange_destroy(m_devEx);
            if (m_localEx) alvrl_local_exchange_destroy(m_localEx);
            m_devEx = NULL;
            m_localEx = NULL;
        }
        for (uint32_t k = 0; k < n; ++k)
            check(rcs[k], "alvrl_integrator_prepass_dist (amdDevices)");
    }

    /* the ranks' collective: RCCL over xGMI between distinct devices, host
       memory for a one-GPU rehearsal (amdRehearseDevices) */
    void ensureExchange() {
        if (m_more.empty() || m_localEx || m_devEx)
            return;
        if (m_rehearse)
            check(alvrl_local_exchange_create((uint32_t) m_devices.size(), &m_localEx), "alvrl_local_exchange_create");
        else
            check(alvrl_device_exchange_create(&m_devices[0], (uint32_t) m_devices.size(), &m_devEx),
                  "alvrl_device_exchange_create");
    }

    void releaseMore() {
        for (size_t k = 0; k < m_more.size(); ++k) {
            (void) hipSetDevice(m_devices[k + 1]);
            if (k < m_moreFb.size() && m_moreFb[k]) (void) hipFree(m_moreFb[k]);
            if (k < m_moreStreams.size() && m_moreStreams[k]) (void) hipStreamDestroy(m_moreStreams[k]);
            alvrl_integrator_destroy(m_more[k]);
        }
        m_more.clear(); m_moreFb.clear(); m_moreStreams.clear(); m_moreRgb.clear();
    }

    /* LiInternal (vrlIntegrator.cpp:398-524) as gather records: the segment
     * of 'ray' and, through a delta BSDF, each delta component's continuation
     * (bRec.component = i, :467-511) with its own weight, throughput and
     * roulette.  A record's depth word is its index in the pixel sample's
     * path tree (record k of sample j: k | j << 16): it keys the gathers'
     * streams, so branches at the same depth draw independently. */
    void appendPath(const RayDifferential &ray, RadianceQueryRecord &rRec, const Spectrum &weight,
            const Spectrum &throughputWithEtaSq, uint32_t sampleIndex, std::vector<alvrl_gather_rec> *recs) const {
        appendPathAt(ray, rRec, weight, throughputWithEtaSq, sampleIndex, recs, recs->size());
    }

    void appendPathAt(const RayDifferential &ray, RadianceQueryRecord &rRec, const Spectrum &weight,
            const Spectrum &throughputWithEtaSq, uint32_t sampleIndex, std::vector<alvrl_gather_rec> *recs,
            size_t first) const {
        if (recs->size() - first >= kMaxPathRecords)
            return;
        if (!rRec.rayIntersect(ray))
            return;   /* :418-423: no contribution (an infinite eye ray's is dropped) */
        const Intersection &its = rRec.its;
        const BSDF *bsdf = its.getBSDF();
        const unsigned int type = bsdf->getType();
        alvrl_gather_rec r;
        std::memset(&r, 0, sizeof(r));
        for (int k = 0; k < 3; ++k) {
            r.o[k] = (float) ray.o[k]; r.d[k] = (float) ray.d[k];
            r.p[k] = (float) its.p[k]; r.n[k] = (float) its.shFrame.n[k];
        }
        const bool smooth = (type & BSDF::ESmooth) != 0;
        /* the gathers' vol->surf term is SmoothDiffuse::eval; any
           other smooth BSDF (plastic, rough or glossy ones) is refused rather
           than approximated by its diffuse reflectance */
        if (smooth && bsdf->getClass()->getName() != "SmoothDiffuse")
            Log(EError, "vrl (amd): a smooth %s BSDF is not supported (the library's vol->surf term is the "
                "smooth diffuse BSDF, diffuse.cpp:110-118)", bsdf->getClass()->getName().c_str());
        put3(r.albedo, smooth ? bsdf->getDiffuseReflectance(its) : Spectrum(0.0f));
        r.flags = ALVRL_REC_HIT | (smooth ? ALVRL_REC_SMOOTH : 0u) | ((type & BSDF::EDelta) ? ALVRL_REC_DELTA : 0u) |
            (rRec.medium && !rRec.medium->getSigmaS().isZero() ? ALVRL_REC_MEDIUM : 0u);
        put3(r.weight, weight);
        r.depth = (uint32_t) (recs->size() - first) | (sampleIndex << 16);
        recs->push_back(r);
        if (!(type & BSDF::EDelta))
            return;   /* no specular chains */
        Spectrum transmittance(1.0f);
        if (rRec.medium) {
            MediumSamplingRecord mRec;
            rRec.medium->eval(Ray(ray, 0, its.t), mRec);
            transmittance = mRec.transmittance;
        }
        if (transmittance.isZero())
            return;
        RadianceQueryRecord rRec2;
        for (int i = 0; i < bsdf->getComponentCount(); ++i) {
            if (!(bsdf->getType(i) & BSDF::EDelta))
                continue;
            BSDFSamplingRecord bRec(rRec.its, rRec.sampler, ERadiance);
            bRec.component = i;
            const Spectrum bsdfWeight = bsdf->sample(bRec, Point2(0.5f));
            if (bsdfWeight.isZero())
                continue;
            Spectrum thr2 = throughputWithEtaSq * transmittance * bsdfWeight * (bRec.eta * bRec.eta);
            const Float maxRR = rRec.depth >= m_specRRdepth ? (Float) 0.98f : (Float) 1.0f;
            const Float rrProb = std::min(maxRR, thr2.max());
            if (rrProb <= 0 || (rrProb < 1 && rRec.nextSample1D() > rrProb))
                continue;
            thr2 /= rrProb;
            rRec2.recursiveQuery(rRec);
            const RayDifferential ray2(rRec.its.p, rRec.its.toWorld(bRec.wo), ray.time);
            if (rRec.its.isMediumTransition())
                rRec2.medium = rRec.its.getTargetMedium(ray2.d);
            appendPathAt(ray2, rRec2, weight * transmittance * bsdfWeight / rrProb, thr2, sampleIndex, recs, first);
        }
    }

    /* "records" mode: every sensor sample's eye path cast by Mitsuba, the
     * block's records gathered on the device in one call */
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
                const uint32_t ownerId = (uint32_t) pos.size();
                pos.push_back(samplePos);
                const size_t before = recs.size();
                appendPath(ray, rRec, Spectrum(1.0f), Spectrum(m_initialSpecularThroughput), (uint32_t) j, &recs);
                for (size_t k = before; k < recs.size(); ++k) {
                    ids.push_back(pid);
                    slice.push_back(sl);
                    owner.push_back(ownerId);
                }
                sampler->advance();
            }
        }
        const uint32_t n = (uint32_t) recs.size();
        std::vector<float> rgb((size_t) 3 * n + 3);
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
    int m_sampleCount = 0;
    hipStream_t m_stream = NULL;
    int m_device = 0;
    bool m_recordsMode = false;
    float m_samplingWeight = -1.0f, m_samplingDensity = 0.0f;
    int m_strategy = ALVRL_STRATEGY_BALANCE, m_channel = 0;
    int m_volVolSamples = 2, m_volSurfSamples = 2;
    bool m_globalCluster = false, m_localRefinement = true, m_shortVrls = true;
    int m_specRRdepth = 100;
    Float m_initialSpecularThroughput = 20;
    std::string m_vrlFile;
    const Medium *m_medium = NULL;
    /* frame mode: the scene (m_desc over m_tris / m_mats / m_emit); records
     * mode: m_tris / m_mats are every shape's triangles (the gathers'
     * occluder set) and m_tdesc over m_ttris / m_tmats / m_temit the VRL
     * tracer's view of the scene */
    alvrl_scene_desc m_desc, m_tdesc;
    std::vector<float> m_tris, m_ttris;
    std::vector<uint32_t> m_mats, m_tmats;
    std::vector<float> m_emit, m_temit;   /* the area emitter's triangles */
    std::vector<float> m_albs, m_talbs;   /* each triangle's diffuse reflectance */
    std::vector<uint32_t> m_p2s;   // the pass's slice of every pixel (column-major); empty: brute force
    int m_width = 0, m_height = 0;
    float *m_fb = NULL;
    bool m_ready = false;
    int m_vrlsID = 0, m_ciID = 0;
    /* amdDevices: m_devices[0] drives m_it / m_fb / m_stream; the others have
     * their own library integrator, framebuffer, stream and host frame */
    std::vector<int> m_devices;
    std::vector<alvrl_integrator *> m_more;
    std::vector<float *> m_moreFb;
    std::vector<hipStream_t> m_moreStreams;
    mutable std::vector<std::vector<float> > m_moreRgb;
    alvrl_local_exchange *m_localEx = NULL;   /* amdRehearseDevices: ranks exchange through host memory */
    alvrl_device_exchange *m_devEx = NULL;     /* distinct devices: RCCL (mask, lists, frame reduce) */
    bool m_rehearse = false;
    /* wakeup: the VRL resource this instance published (the master) and the
     * last one it installed (a render worker) */
    const SerializableObject *m_pubVrls = NULL;
    int64_t m_installedPass = -1;   /* the pass (VRL set, cluster info) wakeup installed last */
    std::mutex m_wakeLock;
    /* the current pass's frame (frame mode) */
    mutable std::vector<float> m_rgb;
    mutable std::mutex m_frameLock;
    mutable std::condition_variable m_frameReady;
    mutable bool m_rendering = false;
    mutable int m_framePass = -1;
    int m_pass = 0;
};

MTS_IMPLEMENT_CLASS_S(AmdVrlSet, false, SerializableObject)
MTS_IMPLEMENT_CLASS_S(AmdClusterInfo, false, SerializableObject)
MTS_IMPLEMENT_CLASS_S(vrlAmdIntegrator, false, ProgressiveMonteCarloIntegrator)
MTS_EXPORT_PLUGIN(vrlAmdIntegrator, "VRL integrator with Adaptive LightSlice on an MI355X (libalvrl)");
MTS_NAMESPACE_END
