/* mock of src/integrators/vrl/VRL.h + vrlTracer.h: the declarations the
 * plugin's records mode uses (VRL's public members, vrlVector's accessors,
 * vrlTracer's constructor and randomWalk, vrlTracer.h:10-15).  Test
 * infrastructure for tests/test_plugin_source.py; see mitsuba/mock.h. */
#pragma once
#include <mitsuba/mock.h>

MTS_NAMESPACE_BEGIN

class VRL : public SerializableObject {
public:
    Spectrum m_power;
    Point m_start;
    Point m_end;
};

class vrlVector : public SerializableObject {
public:
    size_t size() const;
    size_t getParticleCount() const;
    const VRL &operator[](size_t index) const;
};

class vrlTracer : public Object {
public:
    vrlTracer(ref<Sampler> sampler, int maxDepth, int rrDepth);
    ref<vrlVector> randomWalk(const Scene *scene, unsigned int vrlTargetNum, bool shortVrls);
};

MTS_NAMESPACE_END
