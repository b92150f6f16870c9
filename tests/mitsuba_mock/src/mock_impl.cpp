/*
 * mock_impl.cpp -- just enough of Mitsuba 0.x (the declarations of
 * tests/mitsuba_mock/include/mitsuba/mock.h) to load the vrl (amd) plugin
 * (mitsuba_plugin/vrlAmdIntegrator.cpp) and run it in "frame" mode: a smoke
 * box -- perspective camera inside a homogeneous medium, the box as a
 * triangle mesh with a smooth diffuse BSDF holding the medium, one point
 * light -- properties from a "name=value;..." string, the scheduler's
 * resource table, and image blocks that write into one RGB frame.  Test
 * infrastructure (tests/test_gpu_plugin_run.py), not Mitsuba: nothing here
 * is built into libalvrl.so or the plugin.
 *
 * mock_run_frame() plays the parts of Mitsuba's render loop the plugin sees
 * for a progressive render (integrator.cpp, renderproc.cpp): CreateInstance,
 * preprocess, then per pass prepass and renderBlock over 32x32 blocks, and
 * the serialization round trip of a remote worker.  The records-mode entry
 * points (ray casting, BSDF sampling) are not implemented and abort.
 */
#include <mitsuba/mock.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <string>

#include "alvrl.h"
#include "alvrl_host.h"

MTS_NAMESPACE_BEGIN

static void unsupported(const char *what) {
    std::fprintf(stderr, "mitsuba mock: %s is not implemented (frame mode only)\n", what);
    std::abort();
}

/* Log(EError) throws, as Mitsuba's does (the plugin relies on it) */
void mockLog(ELogLevel level, const char *fmt, ...) {
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (level >= EError)
        throw std::runtime_error(buf);
    if (level >= EWarn)
        std::fprintf(stderr, "mock log: %s\n", buf);
}

/* ---- core ---- */
Object::Object() : m_refCount(0) { }
Object::~Object() { }
void Object::incRef() const { ++m_refCount; }
void Object::decRef(bool autoDeallocate) const {
    if (--m_refCount == 0 && autoDeallocate)
        delete this;
}
const Class *Object::getClass() const {
    static Class *c = new Class("Object", false, "");
    return c;
}
std::string Object::toString() const { return getClass()->getName(); }

Class::Class(const std::string &name, bool, const std::string &, void *, void *) : m_name(name) { }
const std::string &Class::getName() const { return m_name; }

SerializableObject::SerializableObject() { }
SerializableObject::SerializableObject(Stream *, InstanceManager *) { }
void SerializableObject::serialize(Stream *, InstanceManager *) const { }
ConfigurableObject::ConfigurableObject(const Properties &) { }
ConfigurableObject::ConfigurableObject() { }
ConfigurableObject::ConfigurableObject(Stream *s, InstanceManager *m) : SerializableObject(s, m) { }
void ConfigurableObject::serialize(Stream *s, InstanceManager *m) const { SerializableObject::serialize(s, m); }

/* Stream: an in-memory byte buffer (the remote worker's round trip) */
struct MemStream : public Stream {
    std::string buf;
    size_t pos;
    MemStream() : pos(0) { }
    void put(const void *p, size_t n) { buf.append((const char *) p, n); }
    void get(void *p, size_t n) {
        if (pos + n > buf.size()) throw std::runtime_error("mock stream: read past the end");
        std::memcpy(p, buf.data() + pos, n);
        pos += n;
    }
};
static MemStream &ms(Stream *s) { return *static_cast<MemStream *>(s); }
void Stream::writeString(const std::string &v) { writeULong(v.size()); ms(this).put(v.data(), v.size()); }
void Stream::writeInt(int v) { ms(this).put(&v, sizeof(v)); }
void Stream::writeUInt(unsigned int v) { ms(this).put(&v, sizeof(v)); }
void Stream::writeULong(uint64_t v) { ms(this).put(&v, sizeof(v)); }
void Stream::writeSingle(float v) { ms(this).put(&v, sizeof(v)); }
void Stream::writeSingleArray(const float *d, size_t n) { ms(this).put(d, n * sizeof(float)); }
void Stream::writeFloat(Float v) { ms(this).put(&v, sizeof(v)); }
void Stream::writeBool(bool v) { char c = v ? 1 : 0; ms(this).put(&c, 1); }
std::string Stream::readString() {
    std::string v((size_t) readULong(), '\0');
    if (!v.empty()) ms(this).get(&v[0], v.size());
    return v;
}
int Stream::readInt() { int v; ms(this).get(&v, sizeof(v)); return v; }
unsigned int Stream::readUInt() { unsigned int v; ms(this).get(&v, sizeof(v)); return v; }
uint64_t Stream::readULong() { uint64_t v; ms(this).get(&v, sizeof(v)); return v; }
float Stream::readSingle() { float v; ms(this).get(&v, sizeof(v)); return v; }
void Stream::readSingleArray(float *d, size_t n) { ms(this).get(d, n * sizeof(float)); }
Float Stream::readFloat() { Float v; ms(this).get(&v, sizeof(v)); return v; }
bool Stream::readBool() { char c; ms(this).get(&c, 1); return c != 0; }

/* Properties (name=value;...) */
static bool findProp(const Properties &p, const std::string &n, std::string *v) {
    std::map<std::string, std::string>::const_iterator it = p.m_values.find(n);
    if (it == p.m_values.end()) return false;
    *v = it->second;
    return true;
}
bool Properties::getBoolean(const std::string &n, bool d) const {
    std::string v;
    return findProp(*this, n, &v) ? (v == "true" || v == "1") : d;
}
int Properties::getInteger(const std::string &n, int d) const {
    std::string v;
    return findProp(*this, n, &v) ? std::atoi(v.c_str()) : d;
}
Float Properties::getFloat(const std::string &n, Float d) const {
    std::string v;
    return findProp(*this, n, &v) ? (Float) std::atof(v.c_str()) : d;
}
std::string Properties::getString(const std::string &n, const std::string &d) const {
    std::string v;
    return findProp(*this, n, &v) ? v : d;
}
std::string Properties::getAsString(const std::string &n) const { return getString(n, ""); }
void Properties::putPropertyNames(std::vector<std::string> &r) const {
    for (std::map<std::string, std::string>::const_iterator it = m_values.begin(); it != m_values.end(); ++it)
        r.push_back(it->first);
}

void ParallelProcess::bindResource(const std::string &, int) { }

Scheduler *Scheduler::getInstance() {
    static Scheduler *s = NULL;
    if (!s) { s = new Scheduler(); s->incRef(); s->m_next = 1; }
    return s;
}
int Scheduler::registerResource(SerializableObject *r) { m_res[m_next] = r; return m_next++; }
bool Scheduler::unregisterResource(int id) { return m_res.erase(id) > 0; }
SerializableObject *Scheduler::getResource(int id, int) {
    std::map<int, ref<SerializableObject> >::iterator it = m_res.find(id);
    return it == m_res.end() ? NULL : it->second.get();
}

/* ---- geometry ---- */
template <typename T> TVector2<T>::TVector2() : x(0), y(0) { }
template <typename T> TVector2<T>::TVector2(T v) : x(v), y(v) { }
template <typename T> TVector2<T>::TVector2(T a, T b) : x(a), y(b) { }
template <typename T> TVector2<T>::TVector2(const TPoint2<T> &p) : x(p.x), y(p.y) { }
template <typename T> TPoint2<T>::TPoint2() : x(0), y(0) { }
template <typename T> TPoint2<T>::TPoint2(T v) : x(v), y(v) { }
template <typename T> TPoint2<T>::TPoint2(T a, T b) : x(a), y(b) { }
template <typename T> template <typename T2> TPoint2<T>::TPoint2(const TPoint2<T2> &p) : x((T) p.x), y((T) p.y) { }
template <typename T> TPoint2<T> TPoint2<T>::operator+(const TVector2<T> &v) const { return TPoint2<T>(x + v.x, y + v.y); }
template struct TVector2<float>;
template struct TVector2<int>;
template struct TPoint2<float>;
template struct TPoint2<int>;
template struct TPoint2<uint8_t>;
template TPoint2<float>::TPoint2(const TPoint2<int> &);
template TPoint2<int>::TPoint2(const TPoint2<uint8_t> &);

Vector::Vector() : x(0), y(0), z(0) { }
Vector::Vector(Float v) : x(v), y(v), z(v) { }
Vector::Vector(Float a, Float b, Float c) : x(a), y(b), z(c) { }
Float Vector::operator[](int i) const { return i == 0 ? x : i == 1 ? y : z; }
Vector Vector::operator-() const { return Vector(-x, -y, -z); }
Vector Vector::operator+(const Vector &v) const { return Vector(x + v.x, y + v.y, z + v.z); }
Vector cross(const Vector &a, const Vector &b) {
    return Vector(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
Float dot(const Vector &a, const Vector &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
Point::Point() : x(0), y(0), z(0) { }
Point::Point(Float v) : x(v), y(v), z(v) { }
Point::Point(Float a, Float b, Float c) : x(a), y(b), z(c) { }
Float Point::operator[](int i) const { return i == 0 ? x : i == 1 ? y : z; }
Point Point::operator+(const Vector &v) const { return Point(x + v.x, y + v.y, z + v.z); }
Vector Point::operator-(const Point &p) const { return Vector(x - p.x, y - p.y, z - p.z); }

Point Transform::operator()(const Point &p) const {
    double r[3];
    for (int i = 0; i < 3; ++i) r[i] = m[i][0] * p.x + m[i][1] * p.y + m[i][2] * p.z + m[i][3];
    return Point((Float) r[0], (Float) r[1], (Float) r[2]);
}
Vector Transform::operator()(const Vector &v) const {
    double r[3];
    for (int i = 0; i < 3; ++i) r[i] = m[i][0] * v.x + m[i][1] * v.y + m[i][2] * v.z;
    return Vector((Float) r[0], (Float) r[1], (Float) r[2]);
}
Transform AnimatedTransform::eval(Float) const { return m_t; }

Ray::Ray() : mint(Epsilon), maxt(1e30f), time(0) { }
Ray::Ray(const Ray &r, Float a, Float b) : o(r.o), mint(a), d(r.d), maxt(b), time(r.time) { }
Ray::Ray(const Point &o_, const Vector &d_, Float t) : o(o_), mint(Epsilon), d(d_), maxt(1e30f), time(t) { }
Ray::Ray(const Point &o_, const Vector &d_, Float a, Float b, Float t) : o(o_), mint(a), d(d_), maxt(b), time(t) { }
Point Ray::operator()(Float t) const { return o + Vector(d.x * t, d.y * t, d.z * t); }
RayDifferential::RayDifferential() { }
RayDifferential::RayDifferential(const Point &p, const Vector &d, Float t) : Ray(p, d, t) { }
RayDifferential::RayDifferential(const Ray &r) : Ray(r) { }

Spectrum::Spectrum() { s[0] = s[1] = s[2] = 0; }
Spectrum::Spectrum(Float v) { s[0] = s[1] = s[2] = v; }
Float Spectrum::operator[](int i) const { return s[i]; }
Float &Spectrum::operator[](int i) { return s[i]; }
Spectrum Spectrum::operator*(const Spectrum &o) const {
    Spectrum r; for (int i = 0; i < 3; ++i) r.s[i] = s[i] * o.s[i]; return r;
}
Spectrum Spectrum::operator*(Float f) const { Spectrum r; for (int i = 0; i < 3; ++i) r.s[i] = s[i] * f; return r; }
Spectrum Spectrum::operator/(Float f) const { Spectrum r; for (int i = 0; i < 3; ++i) r.s[i] = s[i] / f; return r; }
Spectrum &Spectrum::operator/=(Float f) { for (int i = 0; i < 3; ++i) s[i] /= f; return *this; }
Spectrum &Spectrum::operator+=(const Spectrum &o) { for (int i = 0; i < 3; ++i) s[i] += o.s[i]; return *this; }
bool Spectrum::operator==(const Spectrum &o) const { return s[0] == o.s[0] && s[1] == o.s[1] && s[2] == o.s[2]; }
bool Spectrum::operator!=(const Spectrum &o) const { return !(*this == o); }
bool Spectrum::isZero() const { return s[0] == 0 && s[1] == 0 && s[2] == 0; }
Float Spectrum::max() const { return std::max(s[0], std::max(s[1], s[2])); }
void Spectrum::toLinearRGB(Float &r, Float &g, Float &b) const { r = s[0]; g = s[1]; b = s[2]; }
void Spectrum::fromLinearRGB(Float r, Float g, Float b) { s[0] = r; s[1] = g; s[2] = b; }

/* ---- render ---- */
Intersection::Intersection() : t(0), shape(NULL) { }
const BSDF *Intersection::getBSDF() const { return shape ? shape->getBSDF() : NULL; }
Vector Intersection::toWorld(const Vector &) const { unsupported("Intersection::toWorld"); return Vector(); }
bool Intersection::isMediumTransition() const { unsupported("Intersection::isMediumTransition"); return false; }
const Medium *Intersection::getTargetMedium(const Vector &) const { unsupported("Intersection::getTargetMedium"); return NULL; }

void Sampler::generate(const Point2i &) { m_sampleIndex = 0; }
void Sampler::advance() { ++m_sampleIndex; }
size_t Sampler::getSampleCount() const { return m_sampleCount; }
size_t Sampler::getSampleIndex() const { return m_sampleIndex; }

Float PhaseFunction::getMeanCosine() const { return 0.0f; }
const PhaseFunction *Medium::getPhaseFunction() const { return m_phase.get(); }
const Spectrum &Medium::getSigmaA() const { return m_sigmaA; }
const Spectrum &Medium::getSigmaS() const { return m_sigmaS; }

BSDFSamplingRecord::BSDFSamplingRecord(const Intersection &i, Sampler *s, ETransportMode m)
    : its(i), sampler(s), eta(1), mode(m), typeMask(0), component(-1), sampledType(0), sampledComponent(-1) { }
int BSDF::getComponentCount() const { return 1; }
unsigned int BSDF::getType() const { return m_type; }
unsigned int BSDF::getType(int) const { return m_type; }
Spectrum BSDF::getSpecularReflectance(const Intersection &) const { return Spectrum(0.0f); }
Float BSDF::getEta() const { return 1.0f; }

PositionSamplingRecord::PositionSamplingRecord() : pdf(0), object(NULL) { }
PositionSamplingRecord::PositionSamplingRecord(Float) : pdf(0), object(NULL) { }
DirectionSamplingRecord::DirectionSamplingRecord() : pdf(0), measure(EInvalidMeasure) { }
DirectionSamplingRecord::DirectionSamplingRecord(const Vector &d_, EMeasure m) : d(d_), pdf(0), measure(m) { }
unsigned int Emitter::getType() const { return m_type; }
Spectrum Emitter::evalPosition(const PositionSamplingRecord &) const { return Spectrum(0.0f); }

void Shape::samplePosition(PositionSamplingRecord &pRec, const Point2 &sample) const {
    /* a point of the shape's first triangle (what diffuseReflectance needs:
       a position and uv; the smooth diffuse reflectance here is constant) */
    const TriMesh *m = dynamic_cast<const TriMesh *>(this);
    if (!m || m->m_tri.empty()) unsupported("Shape::samplePosition of a non-mesh");
    const Triangle &t = m->m_tri[0];
    const Point &a = m->m_pos[t.idx[0]], &b = m->m_pos[t.idx[1]], &c = m->m_pos[t.idx[2]];
    const Float u = sample.x, v = sample.y * (1 - sample.x);
    pRec.p = a + Vector((b.x - a.x) * u + (c.x - a.x) * v, (b.y - a.y) * u + (c.y - a.y) * v,
                        (b.z - a.z) * u + (c.z - a.z) * v);
    pRec.uv = sample;
    pRec.pdf = 1;
}
ref<TriMesh> Shape::createTriMesh() { return ref<TriMesh>(); }
const BSDF *Shape::getBSDF() const { return m_bsdf.get(); }
bool Shape::isEmitter() const { return m_emitter.get() != NULL; }
const Emitter *Shape::getEmitter() const { return m_emitter.get(); }
const Medium *Shape::getInteriorMedium() const { return m_interior; }
const Medium *Shape::getExteriorMedium() const { return m_exterior; }
std::string Shape::getName() const { return m_name; }

AABB TriMesh::getAABB() const {
    AABB b;
    b.min = Point(1e30f); b.max = Point(-1e30f);
    for (size_t i = 0; i < m_pos.size(); ++i) {
        b.min = Point(std::min(b.min.x, m_pos[i].x), std::min(b.min.y, m_pos[i].y), std::min(b.min.z, m_pos[i].z));
        b.max = Point(std::max(b.max.x, m_pos[i].x), std::max(b.max.y, m_pos[i].y), std::max(b.max.z, m_pos[i].z));
    }
    return b;
}
ref<TriMesh> TriMesh::createTriMesh() { return ref<TriMesh>(this); }
const Point *TriMesh::getVertexPositions() const { return m_pos.empty() ? NULL : &m_pos[0]; }
const Normal *TriMesh::getVertexNormals() const { return m_nrm.empty() ? NULL : &m_nrm[0]; }
bool TriMesh::hasVertexNormals() const { return !m_nrm.empty(); }
const Triangle *TriMesh::getTriangles() const { return m_tri.empty() ? NULL : &m_tri[0]; }
size_t TriMesh::getTriangleCount() const { return m_tri.size(); }

const Vector2i &Film::getSize() const { return m_size; }
const Vector2i &Film::getCropSize() const { return m_size; }
Spectrum Sensor::sampleRayDifferential(RayDifferential &, const Point2 &, const Point2 &, Float) const {
    unsupported("Sensor::sampleRayDifferential");
    return Spectrum();
}
bool Sensor::getSamplePosition(const PositionSamplingRecord &, const DirectionSamplingRecord &, Point2 &) const {
    unsupported("Sensor::getSamplePosition");
    return false;
}
const Film *Sensor::getFilm() const { return m_film.get(); }
const Medium *Sensor::getMedium() const { return m_medium; }
const AnimatedTransform *Sensor::getWorldTransform() const { return m_toWorld.get(); }
Float PerspectiveCamera::getXFov() const { return m_xfov; }

bool Scene::rayIntersect(const Ray &, Intersection &) const { unsupported("Scene::rayIntersect"); return false; }
const AABB &Scene::getAABB() const { return m_aabb; }
const Sensor *Scene::getSensor() const { return m_sensor.get(); }
const ref_vector<Medium> &Scene::getMedia() const { return m_media; }
const ref_vector<Emitter> &Scene::getEmitters() const { return m_emitters; }
const ref_vector<Shape> &Scene::getShapes() const { return m_shapes; }

void ImageBlock::clear() { }
const Point2i &ImageBlock::getOffset() const { return m_offset; }
bool ImageBlock::put(const Point2 &pos, const Spectrum &spec, Float) {
    const int x = (int) std::floor(pos.x), y = (int) std::floor(pos.y);
    float *p = m_frame + 3 * ((size_t) y * m_frameWidth + x);
    p[0] = spec.s[0]; p[1] = spec.s[1]; p[2] = spec.s[2];
    return true;
}

RadianceQueryRecord::RadianceQueryRecord() : type(0), scene(NULL), sampler(NULL), medium(NULL), depth(0) { }
RadianceQueryRecord::RadianceQueryRecord(const Scene *s, Sampler *sm)
    : type(0), scene(s), sampler(sm), medium(NULL), depth(0) { }
void RadianceQueryRecord::newQuery(int t, const Medium *m) { type = t; medium = m; depth = 1; }
void RadianceQueryRecord::recursiveQuery(const RadianceQueryRecord &p) { *this = p; ++depth; }
bool RadianceQueryRecord::rayIntersect(const RayDifferential &) { unsupported("RadianceQueryRecord::rayIntersect"); return false; }
Float RadianceQueryRecord::nextSample1D() { unsupported("RadianceQueryRecord::nextSample1D"); return 0; }
Point2 RadianceQueryRecord::nextSample2D() { unsupported("RadianceQueryRecord::nextSample2D"); return Point2(); }

/* integrator.h: the bases' defaults */
Integrator::Integrator(const Properties &p) : ConfigurableObject(p) { }
Integrator::Integrator(Stream *s, InstanceManager *m) : ConfigurableObject(s, m) { }
bool Integrator::preprocess(const Scene *, RenderQueue *, const RenderJob *, int, int, int) { return true; }
void Integrator::bindUsedResources(ParallelProcess *) const { }
void Integrator::wakeup(ConfigurableObject *, std::map<std::string, SerializableObject *> &) { }
void Integrator::serialize(Stream *s, InstanceManager *m) const { ConfigurableObject::serialize(s, m); }
SamplingIntegrator::SamplingIntegrator(const Properties &p) : Integrator(p) { }
SamplingIntegrator::SamplingIntegrator(Stream *s, InstanceManager *m) : Integrator(s, m) { }
void SamplingIntegrator::renderBlock(const Scene *, const Sensor *, Sampler *, ImageBlock *, const bool &,
                                     const std::vector< TPoint2<uint8_t> > &) const {
    unsupported("SamplingIntegrator::renderBlock");
}
void SamplingIntegrator::serialize(Stream *s, InstanceManager *m) const { Integrator::serialize(s, m); }
MonteCarloIntegrator::MonteCarloIntegrator(const Properties &p) : SamplingIntegrator(p) { }
MonteCarloIntegrator::MonteCarloIntegrator(Stream *s, InstanceManager *m) : SamplingIntegrator(s, m) { }
void MonteCarloIntegrator::serialize(Stream *s, InstanceManager *m) const { SamplingIntegrator::serialize(s, m); }
ProgressiveMonteCarloIntegrator::ProgressiveMonteCarloIntegrator(const Properties &p)
    : MonteCarloIntegrator(p), m_maxPasses(p.getInteger("maxPasses", 1)), m_dumpPasses(false) { }
ProgressiveMonteCarloIntegrator::ProgressiveMonteCarloIntegrator(Stream *s, InstanceManager *m)
    : MonteCarloIntegrator(s, m), m_maxPasses(s->readInt()), m_dumpPasses(s->readBool()) { }
std::string ProgressiveMonteCarloIntegrator::passFileSuffix() { return ""; }
void ProgressiveMonteCarloIntegrator::serialize(Stream *s, InstanceManager *m) const {
    MonteCarloIntegrator::serialize(s, m);
    s->writeInt(m_maxPasses);
    s->writeBool(m_dumpPasses);
}

/* ---- the smoke box ---- */
namespace {

struct MockClassed {
    static const Class *make(const char *name) { return new Class(name, false, ""); }
};

class HomogeneousMedium : public Medium {
public:
    void eval(const Ray &, MediumSamplingRecord &) const { unsupported("HomogeneousMedium::eval"); }
    const Class *getClass() const { static const Class *c = MockClassed::make("HomogeneousMedium"); return c; }
};
class IsotropicPhaseFunction : public PhaseFunction {
public:
    const Class *getClass() const { static const Class *c = MockClassed::make("IsotropicPhaseFunction"); return c; }
};
class SmoothDiffuse : public BSDF {
public:
    Spectrum m_reflectance;
    Spectrum sample(BSDFSamplingRecord &, const Point2 &) const { unsupported("SmoothDiffuse::sample"); return Spectrum(); }
    Spectrum getDiffuseReflectance(const Intersection &) const { return m_reflectance; }
    const Class *getClass() const { static const Class *c = MockClassed::make("SmoothDiffuse"); return c; }
};
class PointEmitter : public Emitter {
public:
    Point m_pos;
    Spectrum m_intensity;
    /* point.cpp:81-91: the position and the power, intensity * 4 pi */
    Spectrum samplePosition(PositionSamplingRecord &pRec, const Point2 &, const Point2 *) const {
        pRec.p = m_pos;
        pRec.pdf = 1.0f;
        return m_intensity * (Float) (4.0 * 3.14159265358979323846);
    }
    const Class *getClass() const { static const Class *c = MockClassed::make("PointEmitter"); return c; }
};
class Box : public TriMesh {
public:
    const Class *getClass() const { static const Class *c = MockClassed::make("TriMesh"); return c; }
};
class Camera : public PerspectiveCamera {
public:
    Spectrum sampleRay(Ray &, const Point2 &, const Point2 &, Float) const { unsupported("Camera::sampleRay"); return Spectrum(); }
    const Class *getClass() const { static const Class *c = MockClassed::make("PerspectiveCamera"); return c; }
};
class IndependentSampler : public Sampler {
public:
    Float next1D() { unsupported("Sampler::next1D"); return 0; }
    Point2 next2D() { unsupported("Sampler::next2D"); return Point2(); }
};

/* the scene alvrl_scene_default describes (the bench's smoke box) */
ref<Scene> makeScene(const alvrl_scene_desc &d) {
    ref<Scene> sc = new Scene();
    ref<HomogeneousMedium> med = new HomogeneousMedium();
    med->m_sigmaS.fromLinearRGB(d.medium.sigma_s[0], d.medium.sigma_s[1], d.medium.sigma_s[2]);
    med->m_sigmaA.fromLinearRGB(d.medium.sigma_a[0], d.medium.sigma_a[1], d.medium.sigma_a[2]);
    med->m_phase = new IsotropicPhaseFunction();
    sc->m_media.push_back(ref<Medium>(med.get()));

    ref<Camera> cam = new Camera();
    cam->m_xfov = d.fov_x_deg;
    cam->m_medium = med.get();
    ref<Film> film = new Film();
    film->m_size = Vector2i(d.width, d.height);
    cam->m_film = film;
    /* toWorld: o = T(0,0,0), target = T(0,0,1), up = T(vector 0,1,0), exact */
    ref<AnimatedTransform> tw = new AnimatedTransform();
    for (int i = 0; i < 3; ++i) {
        tw->m_t.m[i][0] = 0.0;
        tw->m_t.m[i][1] = d.cam_up[i];
        tw->m_t.m[i][2] = (double) d.cam_target[i] - (double) d.cam_origin[i];
        tw->m_t.m[i][3] = d.cam_origin[i];
    }
    cam->m_toWorld = tw;
    sc->m_sensor = ref<Sensor>(cam.get());

    ref<PointEmitter> light = new PointEmitter();
    light->m_type = Emitter::EDeltaPosition;
    light->m_pos = Point(d.light_pos[0], d.light_pos[1], d.light_pos[2]);
    light->m_intensity.fromLinearRGB(d.light_intensity[0], d.light_intensity[1], d.light_intensity[2]);
    sc->m_emitters.push_back(ref<Emitter>(light.get()));

    /* the container: a box mesh, smooth diffuse walls, the medium inside */
    ref<Box> box = new Box();
    box->m_name = "smokebox";
    const float *lo = d.box_min, *hi = d.box_max;
    for (int c = 0; c < 8; ++c)
        box->m_pos.push_back(Point((c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]));
    static const uint32_t faces[6][4] = {{0, 2, 6, 4}, {1, 5, 7, 3}, {0, 4, 5, 1}, {2, 3, 7, 6}, {0, 1, 3, 2}, {4, 6, 7, 5}};
    for (int f = 0; f < 6; ++f) {
        Triangle a, b;
        a.idx[0] = faces[f][0]; a.idx[1] = faces[f][1]; a.idx[2] = faces[f][2];
        b.idx[0] = faces[f][0]; b.idx[1] = faces[f][2]; b.idx[2] = faces[f][3];
        box->m_tri.push_back(a);
        box->m_tri.push_back(b);
    }
    ref<SmoothDiffuse> walls = new SmoothDiffuse();
    walls->m_type = BSDF::EDiffuseReflection;
    walls->m_reflectance.fromLinearRGB(d.albedo[0], d.albedo[1], d.albedo[2]);
    box->m_bsdf = ref<BSDF>(walls.get());
    box->m_interior = med.get();
    box->m_exterior = NULL;
    sc->m_shapes.push_back(ref<Shape>(box.get()));
    sc->m_aabb = box->getAABB();
    return sc;
}

Properties parseProps(const std::string &s) {
    Properties p;
    std::stringstream ss(s);
    std::string kv;
    while (std::getline(ss, kv, ';')) {
        const size_t e = kv.find('=');
        if (e == std::string::npos || e == 0) continue;
        p.m_values[kv.substr(0, e)] = kv.substr(e + 1);
    }
    return p;
}

thread_local std::string g_err;

}  // namespace

MTS_NAMESPACE_END

extern "C" void *CreateInstance(const mitsuba::Properties &props);
MTS_NAMESPACE_BEGIN
/* the plugin's unserializer (MTS_IMPLEMENT_CLASS_S, class.h:219-222) */
Object *__vrlAmdIntegrator_unSer(Stream *stream, InstanceManager *manager);
MTS_NAMESPACE_END

/* A progressive render of the smoke box (alvrl_scene_default(width, height))
 * through the plugin: CreateInstance(props), preprocess, and `passes` passes
 * of prepass + renderBlock over 32x32 blocks.  `remote` != 0: the last pass
 * is rendered by a second instance made the way a remote worker makes it --
 * the master's serialize into a stream, the unserialization constructor, and
 * wakeup with the master's published "vrls" and "vrlClusterInfo" resources.
 * out_rgb (3 * width * height floats) receives the last pass's frame.
 * Returns 0, or -1 with the message in mock_last_error(). */
extern "C" __attribute__((visibility("default"))) int mock_run_frame(const char *props, int width, int height,
                                                                    int passes, int remote, float *out_rgb) {
    using namespace mitsuba;
    try {
        alvrl_scene_desc d;
        alvrl_scene_default(&d, width, height);
        ref<Scene> scene = makeScene(d);
        Properties p = parseProps(props ? props : "");
        ref<ProgressiveMonteCarloIntegrator> it =
            static_cast<ProgressiveMonteCarloIntegrator *>(CreateInstance(p));
        ref<IndependentSampler> sampler = new IndependentSampler();
        sampler->m_sampleCount = 1;
        sampler->m_sampleIndex = 0;
        Scheduler *sched = Scheduler::getInstance();
        const int samplerID = sched->registerResource(sampler.get());
        if (!it->preprocess(scene.get(), NULL, NULL, 0, 0, samplerID))
            throw std::runtime_error("preprocess returned false");
        const int B = 32;
        for (int pass = 0; pass < passes; ++pass) {
            it->prepass(scene.get(), sampler.get());
            ProgressiveMonteCarloIntegrator *renderer = it.get();
            ref<ProgressiveMonteCarloIntegrator> worker;
            if (remote && pass == passes - 1) {
                /* a remote worker: serialize / unserialize, wakeup with the resources */
                MemStream st;
                it->serialize(&st, NULL);
                worker = static_cast<ProgressiveMonteCarloIntegrator *>(
                    mitsuba::__vrlAmdIntegrator_unSer(&st, NULL));
                std::map<std::string, SerializableObject *> params;
                for (std::map<int, ref<SerializableObject> >::iterator r = sched->m_res.begin(); r != sched->m_res.end(); ++r) {
                    const std::string n = r->second->getClass()->getName();
                    if (n == "AmdVrlSet") params["vrls"] = r->second.get();
                    else if (n == "AmdClusterInfo") params["vrlClusterInfo"] = r->second.get();
                }
                worker->wakeup(scene.get(), params);
                renderer = worker.get();
            }
            for (int y0 = 0; y0 < height; y0 += B)
                for (int x0 = 0; x0 < width; x0 += B) {
                    ref<ImageBlock> blk = new ImageBlock();
                    blk->m_offset = Point2i(x0, y0);
                    blk->m_size = Vector2i(std::min(B, width - x0), std::min(B, height - y0));
                    blk->m_frame = out_rgb;
                    blk->m_frameWidth = width;
                    std::vector< TPoint2<uint8_t> > pts;
                    for (int y = 0; y < blk->m_size.y; ++y)
                        for (int x = 0; x < blk->m_size.x; ++x) pts.push_back(TPoint2<uint8_t>((uint8_t) x, (uint8_t) y));
                    const bool stop = false;
                    renderer->renderBlock(scene.get(), scene->getSensor(), sampler.get(), blk.get(), stop, pts);
                }
        }
        sched->unregisterResource(samplerID);
        return 0;
    } catch (const std::exception &e) {
        mitsuba::g_err = e.what();
        return -1;
    }
}

extern "C" __attribute__((visibility("default"))) const char *mock_last_error() { return mitsuba::g_err.c_str(); }
