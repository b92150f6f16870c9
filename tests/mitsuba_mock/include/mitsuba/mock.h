/*
 * mock.h -- the Mitsuba 0.x declarations that mitsuba_plugin/vrlAmdIntegrator.cpp
 * uses, restated (test infrastructure, not Mitsuba).  tests/test_plugin_source.py
 * compiles the plugin against them; tests/mitsuba_mock/src/mock_impl.cpp
 * implements just enough of them -- a smoke-box scene, properties, the
 * scheduler's resources, image blocks -- for tests/test_gpu_plugin_run.py to
 * load the plugin and run it: preprocess, prepass, renderBlock.  The "mock
 * state" members below hold that implementation's data; they are no part of
 * the interface the plugin sees (it never names them).  Signatures follow the
 * mitsuba-ALVRL headers (include/mitsuba/core/{object,class,cobject,sched,
 * stream,properties}.h, render/{integrator,scene,sensor,film,bsdf,medium,
 * phase,emitter,shape,trimesh,imageblock,records}.h) so that a call or an
 * override that does not match them fails to compile.  Two macros are
 * reproduced exactly because the plugin's buildability depends on them:
 * MTS_IMPLEMENT_CLASS_S (class.h:219-226: `new name(stream, manager)`, so the
 * class must have the unserialization constructor) and MTS_EXPORT_PLUGIN
 * (cobject.h:99-107: `new name(props)`, so it must not be abstract).
 */
#ifndef MITSUBA_MOCK_H
#define MITSUBA_MOCK_H

#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#define MTS_NAMESPACE_BEGIN namespace mitsuba {
#define MTS_NAMESPACE_END }
#define MTS_EXPORT __attribute__((visibility("default")))

MTS_NAMESPACE_BEGIN

typedef float Float;
#define Epsilon 1e-4f
#define ShadowEpsilon 1e-3f
#define INV_PI 0.31830988618379067154f

enum ELogLevel { ETrace = 0, EDebug = 100, EInfo = 200, EWarn = 300, EError = 400 };
void mockLog(ELogLevel level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
#define Log(level, fmt, ...) ::mitsuba::mockLog(level, fmt, ## __VA_ARGS__)
#define SLog(level, fmt, ...) ::mitsuba::mockLog(level, fmt, ## __VA_ARGS__)

class Class;
class Stream;
class InstanceManager;

class Object {
public:
    Object();
    void incRef() const;
    void decRef(bool autoDeallocate = true) const;
    virtual const Class *getClass() const;
    virtual std::string toString() const;
protected:
    virtual ~Object();
public:   /* mock state */
    mutable int m_refCount;
};

template <typename T> class ref {
public:
    ref() : m_ptr(NULL) { }
    ref(T *ptr) : m_ptr(ptr) { if (m_ptr) ((const Object *) m_ptr)->incRef(); }
    ref(const ref &r) : m_ptr(r.m_ptr) { if (m_ptr) ((const Object *) m_ptr)->incRef(); }
    ~ref() { if (m_ptr) ((const Object *) m_ptr)->decRef(); }
    ref &operator=(const ref &r) { return *this = r.m_ptr; }
    ref &operator=(T *ptr) {
        if (ptr) ((const Object *) ptr)->incRef();
        if (m_ptr) ((const Object *) m_ptr)->decRef();
        m_ptr = ptr;
        return *this;
    }
    T *operator->() const { return m_ptr; }
    T &operator*() const { return *m_ptr; }
    operator T *() const { return m_ptr; }
    T *get() const { return m_ptr; }
private:
    T *m_ptr;
};
template <typename T> class ref_vector : public std::vector< ref<T> > { };

class Class {
public:
    Class(const std::string &name, bool abstract, const std::string &superClassName, void *instPtr = NULL,
          void *unSerPtr = NULL);
    const std::string &getName() const;
public:   /* mock state */
    std::string m_name;
};

#define MTS_DECLARE_CLASS() \
    virtual const Class *getClass() const; \
    public: \
    static Class *m_theClass;

#define MTS_IMPLEMENT_CLASS_S(name, abstract, super) \
    Object *__##name ##_unSer(Stream *stream, InstanceManager *manager) { \
        return new name(stream, manager); \
    } \
    Class *name::m_theClass = new Class(#name, abstract, #super, NULL, (void *) &__##name ##_unSer); \
    const Class *name::getClass() const { \
        return m_theClass;\
    }

#define MTS_IMPLEMENT_CLASS(name, abstract, super) \
    Class *name::m_theClass = new Class(#name, abstract, #super, NULL, NULL); \
    const Class *name::getClass() const { \
        return m_theClass;\
    }

class Properties;
#define MTS_EXPORT_PLUGIN(name, descr) \
    extern "C" { \
        void MTS_EXPORT *CreateInstance(const Properties &props) { \
            return new name(props); \
        } \
        const char MTS_EXPORT *GetDescription() { \
            return descr; \
        } \
    }

class Stream : public Object {
public:
    void writeString(const std::string &value);
    void writeInt(int value);
    void writeUInt(unsigned int value);
    void writeULong(uint64_t value);
    void writeSingle(float value);
    void writeSingleArray(const float *data, size_t size);
    void writeFloat(Float value);
    void writeBool(bool value);
    std::string readString();
    int readInt();
    unsigned int readUInt();
    uint64_t readULong();
    float readSingle();
    void readSingleArray(float *data, size_t size);
    Float readFloat();
    bool readBool();
};
class InstanceManager : public Object { };

class SerializableObject : public Object {
public:
    SerializableObject(Stream *stream, InstanceManager *manager);
    virtual void serialize(Stream *stream, InstanceManager *manager) const;
protected:
    SerializableObject();
};

class ConfigurableObject : public SerializableObject {
public:
    virtual void serialize(Stream *stream, InstanceManager *manager) const;
protected:
    ConfigurableObject(const Properties &props);
    ConfigurableObject(Stream *stream, InstanceManager *manager);
    ConfigurableObject();   /* mock: the objects mock_impl.cpp builds directly */
};

class Properties {
public:
    bool getBoolean(const std::string &name, bool defVal) const;
    int getInteger(const std::string &name, int defVal) const;
    Float getFloat(const std::string &name, Float defVal) const;
    std::string getString(const std::string &name, const std::string &defVal) const;
    std::string getAsString(const std::string &name) const;
    void putPropertyNames(std::vector<std::string> &results) const;
public:   /* mock state */
    std::map<std::string, std::string> m_values;
};

class ParallelProcess : public Object {
public:
    virtual void bindResource(const std::string &name, int id);
};

class Scheduler : public Object {
public:
    static Scheduler *getInstance();
    int registerResource(SerializableObject *resource);
    bool unregisterResource(int id);
    SerializableObject *getResource(int id, int coreIndex = -1);
public:   /* mock state */
    std::map<int, ref<SerializableObject> > m_res;
    int m_next;
};

/* ---- geometry ---- */
template <typename T> struct TPoint2;
template <typename T> struct TVector2 {
    T x, y;
    TVector2();
    explicit TVector2(T v);
    TVector2(T x, T y);
    explicit TVector2(const TPoint2<T> &p);
};
template <typename T> struct TPoint2 {
    T x, y;
    TPoint2();
    explicit TPoint2(T v);
    TPoint2(T x, T y);
    template <typename T2> explicit TPoint2(const TPoint2<T2> &p);
    TPoint2 operator+(const TVector2<T> &v) const;
};
typedef TPoint2<Float> Point2;
typedef TPoint2<int> Point2i;
typedef TVector2<Float> Vector2;
typedef TVector2<int> Vector2i;

struct Vector {
    Float x, y, z;
    Vector();
    explicit Vector(Float v);
    Vector(Float x, Float y, Float z);
    Float operator[](int i) const;
    Vector operator-() const;
    Vector operator+(const Vector &v) const;
};
struct Normal : public Vector { };
Vector cross(const Vector &a, const Vector &b);
Float dot(const Vector &a, const Vector &b);
struct Point {
    Float x, y, z;
    Point();
    explicit Point(Float v);
    Point(Float x, Float y, Float z);
    Float operator[](int i) const;
    Point operator+(const Vector &v) const;
    Vector operator-(const Point &p) const;
};
struct Frame {
    Vector s, t;
    Normal n;
};
struct AABB {
    Point min, max;
};
struct Transform {
    Point operator()(const Point &p) const;
    Vector operator()(const Vector &v) const;
    /* mock state: an affine map, evaluated in double */
    double m[3][4];
};
class AnimatedTransform : public Object {
public:
    Transform eval(Float t) const;
public:   /* mock state */
    Transform m_t;
};

struct Ray {
    Point o;
    Float mint;
    Vector d;
    Float maxt;
    Float time;
    Ray();
    Ray(const Ray &ray, Float mint, Float maxt);
    Ray(const Point &o, const Vector &d, Float time);
    Ray(const Point &o, const Vector &d, Float mint, Float maxt, Float time);
    Point operator()(Float t) const;
};
struct RayDifferential : public Ray {
    RayDifferential();
    RayDifferential(const Point &p, const Vector &d, Float time);
    explicit RayDifferential(const Ray &ray);
};

class Spectrum {
public:
    Spectrum();
    explicit Spectrum(Float v);
    Float operator[](int i) const;
    Float &operator[](int i);
    Spectrum operator*(const Spectrum &s) const;
    Spectrum operator*(Float f) const;
    Spectrum operator/(Float f) const;
    Spectrum &operator/=(Float f);
    Spectrum &operator+=(const Spectrum &s);
    bool operator==(const Spectrum &s) const;
    bool operator!=(const Spectrum &s) const;
    bool isZero() const;
    Float max() const;
    void toLinearRGB(Float &r, Float &g, Float &b) const;
    void fromLinearRGB(Float r, Float g, Float b);
public:   /* mock state */
    Float s[3];
};

/* ---- render ---- */
class Scene;
class Sampler;
class Medium;
class BSDF;
class Shape;
class TriMesh;
class RenderQueue;
class RenderJob;

enum ETransportMode { ERadiance = 0, EImportance = 1 };

struct Intersection {
    Float t;
    Point p;
    Frame geoFrame;
    Frame shFrame;
    Point2 uv;
    const Shape *shape;
    Intersection();
    const BSDF *getBSDF() const;
    Vector toWorld(const Vector &v) const;
    bool isMediumTransition() const;
    const Medium *getTargetMedium(const Vector &d) const;
};

class Sampler : public ConfigurableObject {
public:
    virtual void generate(const Point2i &offset);
    virtual void advance();
    virtual Float next1D() = 0;
    virtual Point2 next2D() = 0;
    size_t getSampleCount() const;
    size_t getSampleIndex() const;
public:   /* mock state */
    size_t m_sampleCount, m_sampleIndex;
};

struct MediumSamplingRecord {
    Float t;
    Point p;
    Spectrum transmittance;
    Spectrum sigmaA, sigmaS;
    Float pdfSuccess, pdfFailure;
};

class PhaseFunction : public ConfigurableObject {
public:
    virtual Float getMeanCosine() const;
};

class Medium : public ConfigurableObject {
public:
    virtual void eval(const Ray &ray, MediumSamplingRecord &mRec) const = 0;
    const PhaseFunction *getPhaseFunction() const;
    const Spectrum &getSigmaA() const;
    const Spectrum &getSigmaS() const;
public:   /* mock state */
    Spectrum m_sigmaA, m_sigmaS;
    ref<PhaseFunction> m_phase;
};

struct BSDFSamplingRecord {
    BSDFSamplingRecord(const Intersection &its, Sampler *sampler, ETransportMode mode = ERadiance);
    const Intersection &its;
    Sampler *sampler;
    Vector wi, wo;
    Float eta;
    ETransportMode mode;
    unsigned int typeMask;
    int component;
    unsigned int sampledType;
    int sampledComponent;
};

class BSDF : public ConfigurableObject {
public:
    enum EBSDFType {
        ENull = 0x00001, EDiffuseReflection = 0x00002, EDiffuseTransmission = 0x00004,
        EGlossyReflection = 0x00008, EGlossyTransmission = 0x00010, EDeltaReflection = 0x00020,
        EDeltaTransmission = 0x00040, EDelta1DReflection = 0x00080, EDelta1DTransmission = 0x00100
    };
    enum ETypeCombinations {
        EReflection = EDiffuseReflection | EDeltaReflection | EDelta1DReflection | EGlossyReflection,
        ETransmission = EDiffuseTransmission | EDeltaTransmission | EDelta1DTransmission | EGlossyTransmission | ENull,
        EDiffuse = EDiffuseReflection | EDiffuseTransmission,
        EGlossy = EGlossyReflection | EGlossyTransmission,
        ESmooth = EDiffuse | EGlossy,
        EDelta = ENull | EDeltaReflection | EDeltaTransmission,
        EDelta1D = EDelta1DReflection | EDelta1DTransmission,
        EAll = ESmooth | EDelta | EDelta1D
    };
    int getComponentCount() const;
    unsigned int getType() const;
    unsigned int getType(int component) const;
    virtual Spectrum sample(BSDFSamplingRecord &bRec, const Point2 &sample) const = 0;
    virtual Spectrum getDiffuseReflectance(const Intersection &its) const = 0;
    virtual Spectrum getSpecularReflectance(const Intersection &its) const;
    virtual Float getEta() const;
public:   /* mock state */
    unsigned int m_type;
};

/* render/common.h:56-69 */
enum EMeasure { EInvalidMeasure = 0, ESolidAngle = 1, ELength = 2, EArea = 3, EDiscrete = 4 };

struct PositionSamplingRecord {
    Point p;
    Normal n;
    Point2 uv;
    Float pdf;
    const Object *object;
    PositionSamplingRecord();
    PositionSamplingRecord(Float time);
};

/* render/common.h:164-218 */
struct DirectionSamplingRecord {
    Vector d;
    Float pdf;
    EMeasure measure;
    DirectionSamplingRecord();
    DirectionSamplingRecord(const Vector &d, EMeasure measure = ESolidAngle);
};

class Emitter : public ConfigurableObject {
public:
    enum EEmitterType { EDeltaDirection = 0x01, EDeltaPosition = 0x02, EOnSurface = 0x04 };
    unsigned int getType() const;
    virtual Spectrum samplePosition(PositionSamplingRecord &pRec, const Point2 &sample,
                                    const Point2 *extra = NULL) const = 0;
    /* render/emitter.h: the spatial part of the emitted radiance */
    virtual Spectrum evalPosition(const PositionSamplingRecord &pRec) const;
public:   /* mock state */
    unsigned int m_type;
};

class Shape : public ConfigurableObject {
public:
    virtual AABB getAABB() const = 0;
    /* render/shape.h:361-362 */
    virtual void samplePosition(PositionSamplingRecord &pRec, const Point2 &sample) const;
    virtual ref<TriMesh> createTriMesh();
    const BSDF *getBSDF() const;
    /* render/shape.h: the attached area emitter */
    bool isEmitter() const;
    const Emitter *getEmitter() const;
    const Medium *getInteriorMedium() const;
    const Medium *getExteriorMedium() const;
    virtual std::string getName() const;
public:   /* mock state */
    ref<BSDF> m_bsdf;
    ref<Emitter> m_emitter;
    const Medium *m_interior, *m_exterior;
    std::string m_name;
};

struct Triangle {
    uint32_t idx[3];
};

class TriMesh : public Shape {
public:
    AABB getAABB() const;
    ref<TriMesh> createTriMesh();
    const Point *getVertexPositions() const;
    const Normal *getVertexNormals() const;
    bool hasVertexNormals() const;
    const Triangle *getTriangles() const;
    size_t getTriangleCount() const;
public:   /* mock state */
    std::vector<Point> m_pos;
    std::vector<Normal> m_nrm;
    std::vector<Triangle> m_tri;
};

class Film : public ConfigurableObject {
public:
    const Vector2i &getSize() const;
    const Vector2i &getCropSize() const;
public:   /* mock state */
    Vector2i m_size;
};

class Sensor : public ConfigurableObject {
public:
    virtual Spectrum sampleRay(Ray &ray, const Point2 &samplePosition, const Point2 &apertureSample,
                               Float timeSample) const = 0;
    virtual Spectrum sampleRayDifferential(RayDifferential &ray, const Point2 &samplePosition,
                                           const Point2 &apertureSample, Float timeSample) const;
    /* render/sensor.h:265-266 */
    virtual bool getSamplePosition(const PositionSamplingRecord &pRec, const DirectionSamplingRecord &dRec,
                                   Point2 &position) const;
    const Film *getFilm() const;
    const Medium *getMedium() const;
    const AnimatedTransform *getWorldTransform() const;
public:   /* mock state */
    ref<Film> m_film;
    const Medium *m_medium;
    ref<AnimatedTransform> m_toWorld;
};

class PerspectiveCamera : public Sensor {
public:
    Float getXFov() const;
public:   /* mock state */
    Float m_xfov;
};

class Scene : public ConfigurableObject {
public:
    bool rayIntersect(const Ray &ray, Intersection &its) const;
    const AABB &getAABB() const;
    const Sensor *getSensor() const;
    const ref_vector<Medium> &getMedia() const;
    const ref_vector<Emitter> &getEmitters() const;
    const ref_vector<Shape> &getShapes() const;
public:   /* mock state */
    AABB m_aabb;
    ref<Sensor> m_sensor;
    ref_vector<Medium> m_media;
    ref_vector<Emitter> m_emitters;
    ref_vector<Shape> m_shapes;
};

class ImageBlock : public Object {
public:
    void clear();
    const Point2i &getOffset() const;
    bool put(const Point2 &pos, const Spectrum &spec, Float alpha);
public:   /* mock state: puts land in an RGB frame of width m_frameWidth */
    Point2i m_offset;
    Vector2i m_size;
    float *m_frame;
    int m_frameWidth;
};

struct RadianceQueryRecord {
    enum ERadianceQuery {
        EEmittedRadiance = 0x0001, ESubsurfaceRadiance = 0x0002, EDirectSurfaceRadiance = 0x0004,
        EIndirectSurfaceRadiance = 0x0008, ECausticRadiance = 0x0010, EDirectMediumRadiance = 0x0020,
        EIndirectMediumRadiance = 0x0040, EDistance = 0x0080, EOpacity = 0x0100, EIntersection = 0x0200,
        ERadianceNoEmission = ESubsurfaceRadiance | EDirectSurfaceRadiance | EIndirectSurfaceRadiance |
            ECausticRadiance | EDirectMediumRadiance | EIndirectMediumRadiance,
        ERadiance = ERadianceNoEmission | EEmittedRadiance,
        ESensorRay = ERadiance | EOpacity
    };
    RadianceQueryRecord();
    RadianceQueryRecord(const Scene *scene, Sampler *sampler);
    void newQuery(int typeMask, const Medium *medium);
    void recursiveQuery(const RadianceQueryRecord &parent);
    bool rayIntersect(const RayDifferential &ray);
    Float nextSample1D();
    Point2 nextSample2D();
    int type;
    const Scene *scene;
    Sampler *sampler;
    const Medium *medium;
    int depth;
    Intersection its;
};

class Integrator : public ConfigurableObject {
public:
    virtual bool preprocess(const Scene *scene, RenderQueue *queue, const RenderJob *job, int sceneResID,
                            int sensorResID, int samplerResID);
    virtual void bindUsedResources(ParallelProcess *proc) const;
    virtual void wakeup(ConfigurableObject *parent, std::map<std::string, SerializableObject *> &params);
    void serialize(Stream *stream, InstanceManager *manager) const;
protected:
    Integrator(const Properties &props);
    Integrator(Stream *stream, InstanceManager *manager);
};

class SamplingIntegrator : public Integrator {
public:
    virtual Spectrum Li(const RayDifferential &ray, RadianceQueryRecord &rRec) const = 0;
    virtual void renderBlock(const Scene *scene, const Sensor *sensor, Sampler *sampler, ImageBlock *block,
                             const bool &stop, const std::vector< TPoint2<uint8_t> > &points) const;
    void serialize(Stream *stream, InstanceManager *manager) const;
protected:
    SamplingIntegrator(const Properties &props);
    SamplingIntegrator(Stream *stream, InstanceManager *manager);
};

class MonteCarloIntegrator : public SamplingIntegrator {
public:
    void serialize(Stream *stream, InstanceManager *manager) const;
protected:
    MonteCarloIntegrator(const Properties &props);
    MonteCarloIntegrator(Stream *stream, InstanceManager *manager);
};

/* the fork's progressive integrator (include/mitsuba/render/integrator.h:483-511) */
class ProgressiveMonteCarloIntegrator : public MonteCarloIntegrator {
public:
    virtual bool prepass(const Scene *scene, Sampler *sampler) = 0;
    virtual std::string passFileSuffix();
    void serialize(Stream *stream, InstanceManager *manager) const;
protected:
    ProgressiveMonteCarloIntegrator(const Properties &props);
    ProgressiveMonteCarloIntegrator(Stream *stream, InstanceManager *manager);
    virtual ~ProgressiveMonteCarloIntegrator() { }
    int m_maxPasses;
    bool m_dumpPasses;
};

MTS_NAMESPACE_END

#endif
