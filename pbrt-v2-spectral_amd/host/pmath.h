// pmath.h -- host-side geometry/transform library for the MI355X spectral path tracer.
//
// Arithmetic is a restatement of the reference's core/geometry.h, core/transform.{h,cpp}
// and core/quaternion.cpp: every expression keeps the reference's operand order and
// float/double promotions so that scene set-up (camera matrices, object-to-world
// transforms, Loop-subdivided vertices) is bit-identical to what the reference builds.
// Compile with -ffp-contract=off.
#pragma once
#include <cmath>
#include <cstring>
#include <cstdint>
#include <algorithm>

namespace pbrtamd {

static const float kPi = 3.14159265358979323846f;         // pbrt.h:189 (float literal)
static const float kInvPi = 0.31830988618379067154f;
static const float kInvTwoPi = 0.15915494309189533577f;
static const float kOneMinusEps = 0x1.fffffep-1f;        // montecarlo.h:40

template <class T> inline T pmin(T a, T b) { return (b < a) ? b : a; }   // std::min
template <class T> inline T pmax(T a, T b) { return (a < b) ? b : a; }   // std::max
inline float Lerp(float t, float a, float b) { return (1.f - t) * a + t * b; }
inline float Clamp(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
inline int Floor2Int(float v) { return (int)floorf(v); }
inline int Ceil2Int(float v) { return (int)ceilf(v); }
inline float Radians(float deg) { return ((float)kPi / 180.f) * deg; }
inline uint32_t RoundUpPow2(uint32_t v) {
    v--; v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16; return v + 1;
}

// Vector / Point / Normal share storage; the operations that differ between them
// (transforms) are separate functions.
struct V3 {
    float x = 0.f, y = 0.f, z = 0.f;
    V3() {}
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    float operator[](int i) const { return (&x)[i]; }
    float &operator[](int i) { return (&x)[i]; }
    bool operator==(const V3 &o) const { return x == o.x && y == o.y && z == o.z; }
    bool operator!=(const V3 &o) const { return !(*this == o); }
};
inline V3 operator+(const V3 &a, const V3 &b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(const V3 &a, const V3 &b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator-(const V3 &a) { return V3(-a.x, -a.y, -a.z); }
// Vector::operator*(float f) returns (f*x, f*y, f*z); Point::operator* likewise.
inline V3 operator*(const V3 &a, float f) { return V3(f * a.x, f * a.y, f * a.z); }
inline V3 operator*(float f, const V3 &a) { return V3(f * a.x, f * a.y, f * a.z); }
// Vector::operator/ multiplies by the reciprocal (geometry.h:84-88)
inline V3 operator/(const V3 &a, float f) { float inv = 1.f / f; return V3(a.x * inv, a.y * inv, a.z * inv); }
inline V3 &operator+=(V3 &a, const V3 &b) { a.x += b.x; a.y += b.y; a.z += b.z; return a; }
inline V3 &operator*=(V3 &a, float f) { a.x *= f; a.y *= f; a.z *= f; return a; }
inline float Dot(const V3 &a, const V3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float AbsDot(const V3 &a, const V3 &b) { return fabsf(Dot(a, b)); }
inline float LengthSquared(const V3 &a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline float Length(const V3 &a) { return sqrtf(LengthSquared(a)); }
inline V3 Normalize(const V3 &a) { return a / Length(a); }
// Cross is evaluated in double and rounded once to float per component (geometry.h:461-468)
inline V3 Cross(const V3 &a, const V3 &b) {
    double ax = a.x, ay = a.y, az = a.z, bx = b.x, by = b.y, bz = b.z;
    return V3((float)((ay * bz) - (az * by)), (float)((az * bx) - (ax * bz)), (float)((ax * by) - (ay * bx)));
}
inline float DistanceSquared(const V3 &a, const V3 &b) { return LengthSquared(a - b); }
inline V3 Faceforward(const V3 &n, const V3 &v) { return (Dot(n, v) < 0.f) ? -n : n; }
inline void CoordinateSystem(const V3 &v1, V3 *v2, V3 *v3) {
    if (fabsf(v1.x) > fabsf(v1.y)) {
        float invLen = 1.f / sqrtf(v1.x * v1.x + v1.z * v1.z);
        *v2 = V3(-v1.z * invLen, 0.f, v1.x * invLen);
    } else {
        float invLen = 1.f / sqrtf(v1.y * v1.y + v1.z * v1.z);
        *v2 = V3(0.f, v1.z * invLen, -v1.y * invLen);
    }
    *v3 = Cross(v1, *v2);
}

struct BBox {
    V3 pMin{INFINITY, INFINITY, INFINITY}, pMax{-INFINITY, -INFINITY, -INFINITY};
    BBox() {}
    explicit BBox(const V3 &p) : pMin(p), pMax(p) {}
    BBox(const V3 &a, const V3 &b)
        : pMin(pmin(a.x, b.x), pmin(a.y, b.y), pmin(a.z, b.z)), pMax(pmax(a.x, b.x), pmax(a.y, b.y), pmax(a.z, b.z)) {}
    float SurfaceArea() const { V3 d = pMax - pMin; return 2.f * (d.x * d.y + d.x * d.z + d.y * d.z); }
    int MaximumExtent() const {
        V3 d = pMax - pMin;
        if (d.x > d.y && d.x > d.z) return 0;
        else if (d.y > d.z) return 1;
        return 2;
    }
};
inline BBox Union(const BBox &b, const V3 &p) {
    BBox r = b;
    r.pMin.x = pmin(b.pMin.x, p.x); r.pMin.y = pmin(b.pMin.y, p.y); r.pMin.z = pmin(b.pMin.z, p.z);
    r.pMax.x = pmax(b.pMax.x, p.x); r.pMax.y = pmax(b.pMax.y, p.y); r.pMax.z = pmax(b.pMax.z, p.z);
    return r;
}
inline BBox Union(const BBox &b, const BBox &c) {
    BBox r;
    r.pMin.x = pmin(b.pMin.x, c.pMin.x); r.pMin.y = pmin(b.pMin.y, c.pMin.y); r.pMin.z = pmin(b.pMin.z, c.pMin.z);
    r.pMax.x = pmax(b.pMax.x, c.pMax.x); r.pMax.y = pmax(b.pMax.y, c.pMax.y); r.pMax.z = pmax(b.pMax.z, c.pMax.z);
    return r;
}

struct M4 {
    float m[4][4];
    M4() { memset(m, 0, sizeof(m)); m[0][0] = m[1][1] = m[2][2] = m[3][3] = 1.f; }
    M4(float t00, float t01, float t02, float t03, float t10, float t11, float t12, float t13,
       float t20, float t21, float t22, float t23, float t30, float t31, float t32, float t33) {
        m[0][0] = t00; m[0][1] = t01; m[0][2] = t02; m[0][3] = t03;
        m[1][0] = t10; m[1][1] = t11; m[1][2] = t12; m[1][3] = t13;
        m[2][0] = t20; m[2][1] = t21; m[2][2] = t22; m[2][3] = t23;
        m[3][0] = t30; m[3][1] = t31; m[3][2] = t32; m[3][3] = t33;
    }
    bool operator==(const M4 &o) const {
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) if (m[i][j] != o.m[i][j]) return false;
        return true;
    }
    bool operator!=(const M4 &o) const { return !(*this == o); }
};
inline M4 Transpose(const M4 &a) {
    return M4(a.m[0][0], a.m[1][0], a.m[2][0], a.m[3][0], a.m[0][1], a.m[1][1], a.m[2][1], a.m[3][1],
              a.m[0][2], a.m[1][2], a.m[2][2], a.m[3][2], a.m[0][3], a.m[1][3], a.m[2][3], a.m[3][3]);
}
inline M4 Mul(const M4 &a, const M4 &b) {
    M4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j] + a.m[i][3] * b.m[3][j];
    return r;
}
M4 Inverse(const M4 &m);   // Gauss-Jordan, transform.cpp:68-130

struct Xform {
    M4 m, mInv;
    Xform() {}
    explicit Xform(const M4 &a);           // computes inverse
    Xform(const M4 &a, const M4 &ai) : m(a), mInv(ai) {}
    bool operator==(const Xform &o) const { return m == o.m && mInv == o.mInv; }
    bool operator!=(const Xform &o) const { return !(*this == o); }
    // Transform::operator< compares only m (transform.h:112-119) -- used by the cache
    bool operator<(const Xform &t2) const {
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                if (m.m[i][j] < t2.m.m[i][j]) return true;
                if (m.m[i][j] > t2.m.m[i][j]) return false;
            }
        return false;
    }
    bool IsIdentity() const { return m == M4(); }
    // Point (transform.h:184-194): divide only if w != 1
    V3 Point(const V3 &p) const {
        float x = p.x, y = p.y, z = p.z;
        float xp = m.m[0][0] * x + m.m[0][1] * y + m.m[0][2] * z + m.m[0][3];
        float yp = m.m[1][0] * x + m.m[1][1] * y + m.m[1][2] * z + m.m[1][3];
        float zp = m.m[2][0] * x + m.m[2][1] * y + m.m[2][2] * z + m.m[2][3];
        float wp = m.m[3][0] * x + m.m[3][1] * y + m.m[3][2] * z + m.m[3][3];
        if (wp == 1.) return V3(xp, yp, zp);
        float inv = 1.f / wp;
        return V3(inv * xp, inv * yp, inv * zp);   // Point::operator/ : inv*x
    }
    V3 Vector(const V3 &v) const {
        float x = v.x, y = v.y, z = v.z;
        return V3(m.m[0][0] * x + m.m[0][1] * y + m.m[0][2] * z, m.m[1][0] * x + m.m[1][1] * y + m.m[1][2] * z,
                  m.m[2][0] * x + m.m[2][1] * y + m.m[2][2] * z);
    }
    V3 Normal(const V3 &n) const {
        float x = n.x, y = n.y, z = n.z;
        return V3(mInv.m[0][0] * x + mInv.m[1][0] * y + mInv.m[2][0] * z,
                  mInv.m[0][1] * x + mInv.m[1][1] * y + mInv.m[2][1] * z,
                  mInv.m[0][2] * x + mInv.m[1][2] * y + mInv.m[2][2] * z);
    }
    BBox operator()(const BBox &b) const;   // transform.cpp:248-259
    bool SwapsHandedness() const;
};
inline Xform Inverse(const Xform &t) { return Xform(t.mInv, t.m); }
inline Xform operator*(const Xform &a, const Xform &b) { return Xform(Mul(a.m, b.m), Mul(b.mInv, a.mInv)); }
Xform Translate(const V3 &d);
Xform Scale(float x, float y, float z);
Xform Rotate(float angle, const V3 &axis);
Xform LookAt(const V3 &pos, const V3 &look, const V3 &up);
Xform Perspective(float fov, float n, float f);

struct Quat { V3 v{0.f, 0.f, 0.f}; float w = 1.f; };
Quat QuatFromXform(const Xform &t);
Xform QuatToXform(const Quat &q);
Quat Slerp(float t, const Quat &a, const Quat &b);

// AnimatedTransform (transform.h:281-311, transform.cpp:313-397)
struct AnimXform {
    float startTime = 0.f, endTime = 1.f;
    Xform start, end;
    bool animated = false;
    V3 T[2];
    Quat R[2];
    M4 S[2];
    AnimXform() {}
    AnimXform(const Xform &a, float t0, const Xform &b, float t1);
    void Interpolate(float time, Xform *t) const;
    BBox MotionBounds(const BBox &b, bool useInverse) const;
};
void Decompose(const M4 &m, V3 *T, Quat *R, M4 *S);

}  // namespace pbrtamd
