// pmath.cpp -- transform construction; restates core/transform.cpp and core/quaternion.cpp.
#include "pmath.h"
#include <utility>

namespace pbrtamd {

// transform.cpp:68-130 (Gauss-Jordan with full pivoting, float)
M4 Inverse(const M4 &m) {
    int indxc[4], indxr[4];
    int ipiv[4] = {0, 0, 0, 0};
    float minv[4][4];
    memcpy(minv, m.m, 4 * 4 * sizeof(float));
    for (int i = 0; i < 4; i++) {
        int irow = -1, icol = -1;
        float big = 0.;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] != 1) {
                for (int k = 0; k < 4; k++) {
                    if (ipiv[k] == 0) {
                        if (fabsf(minv[j][k]) >= big) {
                            big = float(fabsf(minv[j][k]));
                            irow = j;
                            icol = k;
                        }
                    }
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) std::swap(minv[irow][k], minv[icol][k]);
        indxr[i] = irow;
        indxc[i] = icol;
        float pivinv = 1.f / minv[icol][icol];
        minv[icol][icol] = 1.f;
        for (int j = 0; j < 4; j++) minv[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j != icol) {
                float save = minv[j][icol];
                minv[j][icol] = 0;
                for (int k = 0; k < 4; k++) minv[j][k] -= minv[icol][k] * save;
            }
        }
    }
    for (int j = 3; j >= 0; j--) {
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) std::swap(minv[k][indxr[j]], minv[k][indxc[j]]);
    }
    M4 r;
    memcpy(r.m, minv, sizeof(minv));
    return r;
}

Xform::Xform(const M4 &a) : m(a), mInv(Inverse(a)) {}

BBox Xform::operator()(const BBox &b) const {
    const Xform &M = *this;
    BBox ret(M.Point(V3(b.pMin.x, b.pMin.y, b.pMin.z)));
    ret = Union(ret, M.Point(V3(b.pMax.x, b.pMin.y, b.pMin.z)));
    ret = Union(ret, M.Point(V3(b.pMin.x, b.pMax.y, b.pMin.z)));
    ret = Union(ret, M.Point(V3(b.pMin.x, b.pMin.y, b.pMax.z)));
    ret = Union(ret, M.Point(V3(b.pMin.x, b.pMax.y, b.pMax.z)));
    ret = Union(ret, M.Point(V3(b.pMax.x, b.pMax.y, b.pMin.z)));
    ret = Union(ret, M.Point(V3(b.pMax.x, b.pMin.y, b.pMax.z)));
    ret = Union(ret, M.Point(V3(b.pMax.x, b.pMax.y, b.pMax.z)));
    return ret;
}

bool Xform::SwapsHandedness() const {
    float det = ((m.m[0][0] * (m.m[1][1] * m.m[2][2] - m.m[1][2] * m.m[2][1])) -
                 (m.m[0][1] * (m.m[1][0] * m.m[2][2] - m.m[1][2] * m.m[2][0])) +
                 (m.m[0][2] * (m.m[1][0] * m.m[2][1] - m.m[1][1] * m.m[2][0])));
    return det < 0.f;
}

Xform Translate(const V3 &d) {
    M4 m(1, 0, 0, d.x, 0, 1, 0, d.y, 0, 0, 1, d.z, 0, 0, 0, 1);
    M4 mi(1, 0, 0, -d.x, 0, 1, 0, -d.y, 0, 0, 1, -d.z, 0, 0, 0, 1);
    return Xform(m, mi);
}
Xform Scale(float x, float y, float z) {
    M4 m(x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0, 0, 0, 0, 1);
    M4 mi(1.f / x, 0, 0, 0, 0, 1.f / y, 0, 0, 0, 0, 1.f / z, 0, 0, 0, 0, 1);
    return Xform(m, mi);
}
// transform.cpp:201-222
Xform Rotate(float angle, const V3 &axis) {
    V3 a = Normalize(axis);
    float s = sinf(Radians(angle));
    float c = cosf(Radians(angle));
    M4 m;
    m.m[0][0] = a.x * a.x + (1.f - a.x * a.x) * c;
    m.m[0][1] = a.x * a.y * (1.f - c) - a.z * s;
    m.m[0][2] = a.x * a.z * (1.f - c) + a.y * s;
    m.m[0][3] = 0;
    m.m[1][0] = a.x * a.y * (1.f - c) + a.z * s;
    m.m[1][1] = a.y * a.y + (1.f - a.y * a.y) * c;
    m.m[1][2] = a.y * a.z * (1.f - c) - a.x * s;
    m.m[1][3] = 0;
    m.m[2][0] = a.x * a.z * (1.f - c) - a.y * s;
    m.m[2][1] = a.y * a.z * (1.f - c) + a.x * s;
    m.m[2][2] = a.z * a.z + (1.f - a.z * a.z) * c;
    m.m[2][3] = 0;
    m.m[3][0] = 0; m.m[3][1] = 0; m.m[3][2] = 0; m.m[3][3] = 1;
    return Xform(m, Transpose(m));
}
// transform.cpp:225-245
Xform LookAt(const V3 &pos, const V3 &look, const V3 &up) {
    M4 m;
    m.m[0][3] = pos.x; m.m[1][3] = pos.y; m.m[2][3] = pos.z; m.m[3][3] = 1;
    V3 dir = Normalize(look - pos);
    V3 left = Normalize(Cross(Normalize(up), dir));
    V3 newUp = Cross(dir, left);
    m.m[0][0] = left.x; m.m[1][0] = left.y; m.m[2][0] = left.z; m.m[3][0] = 0.;
    m.m[0][1] = newUp.x; m.m[1][1] = newUp.y; m.m[2][1] = newUp.z; m.m[3][1] = 0.;
    m.m[0][2] = dir.x; m.m[1][2] = dir.y; m.m[2][2] = dir.z; m.m[3][2] = 0.;
    return Xform(Inverse(m), m);
}
// transform.cpp:298-308
Xform Perspective(float fov, float n, float f) {
    M4 persp(1, 0, 0, 0, 0, 1, 0, 0, 0, 0, f / (f - n), -f * n / (f - n), 0, 0, 1, 0);
    float invTanAng = 1.f / tanf(Radians(fov) / 2.f);
    return Scale(invTanAng, invTanAng, 1) * Xform(persp);
}

// quaternion.cpp
Xform QuatToXform(const Quat &q) {
    float xx = q.v.x * q.v.x, yy = q.v.y * q.v.y, zz = q.v.z * q.v.z;
    float xy = q.v.x * q.v.y, xz = q.v.x * q.v.z, yz = q.v.y * q.v.z;
    float wx = q.v.x * q.w, wy = q.v.y * q.w, wz = q.v.z * q.w;
    M4 m;
    m.m[0][0] = 1.f - 2.f * (yy + zz);
    m.m[0][1] = 2.f * (xy + wz);
    m.m[0][2] = 2.f * (xz - wy);
    m.m[1][0] = 2.f * (xy - wz);
    m.m[1][1] = 1.f - 2.f * (xx + zz);
    m.m[1][2] = 2.f * (yz + wx);
    m.m[2][0] = 2.f * (xz + wy);
    m.m[2][1] = 2.f * (yz - wx);
    m.m[2][2] = 1.f - 2.f * (xx + yy);
    return Xform(Transpose(m), m);
}
Quat QuatFromXform(const Xform &t) {
    const M4 &m = t.m;
    Quat q;
    float trace = m.m[0][0] + m.m[1][1] + m.m[2][2];
    if (trace > 0.f) {
        float s = sqrtf((float)(trace + 1.0));
        q.w = s / 2.0f;
        s = 0.5f / s;
        q.v.x = (m.m[2][1] - m.m[1][2]) * s;
        q.v.y = (m.m[0][2] - m.m[2][0]) * s;
        q.v.z = (m.m[1][0] - m.m[0][1]) * s;
    } else {
        const int nxt[3] = {1, 2, 0};
        float qq[3];
        int i = 0;
        if (m.m[1][1] > m.m[0][0]) i = 1;
        if (m.m[2][2] > m.m[i][i]) i = 2;
        int j = nxt[i], k = nxt[j];
        float s = sqrtf((float)((m.m[i][i] - (m.m[j][j] + m.m[k][k])) + 1.0));
        qq[i] = s * 0.5f;
        if (s != 0.f) s = 0.5f / s;
        q.w = (m.m[k][j] - m.m[j][k]) * s;
        qq[j] = (m.m[j][i] + m.m[i][j]) * s;
        qq[k] = (m.m[k][i] + m.m[i][k]) * s;
        q.v = V3(qq[0], qq[1], qq[2]);
    }
    return q;
}
static inline float QDot(const Quat &a, const Quat &b) { return Dot(a.v, b.v) + a.w * b.w; }
static inline Quat QScale(const Quat &a, float f) { Quat r = a; r.v *= f; r.w *= f; return r; }
static inline Quat QAdd(const Quat &a, const Quat &b) { Quat r = a; r.v += b.v; r.w += b.w; return r; }
static inline Quat QSub(const Quat &a, const Quat &b) {
    Quat r = a; r.v = V3(r.v.x - b.v.x, r.v.y - b.v.y, r.v.z - b.v.z); r.w -= b.w; return r;
}
static inline Quat QNormalize(const Quat &q) {
    float d = sqrtf(QDot(q, q));
    Quat r = q;   // Quaternion::operator/ -> Vector::operator/= (reciprocal) and w /= f
    float inv = 1.f / d;
    r.v = V3(r.v.x * inv, r.v.y * inv, r.v.z * inv);
    r.w /= d;
    return r;
}
Quat Slerp(float t, const Quat &q1, const Quat &q2) {
    float cosTheta = QDot(q1, q2);
    if (cosTheta > .9995f) return QNormalize(QAdd(QScale(q1, 1.f - t), QScale(q2, t)));
    float theta = acosf(Clamp(cosTheta, -1.f, 1.f));
    float thetap = theta * t;
    Quat qperp = QNormalize(QSub(q2, QScale(q1, cosTheta)));
    return QAdd(QScale(q1, cosf(thetap)), QScale(qperp, sinf(thetap)));
}

// transform.cpp:313-353
void Decompose(const M4 &m, V3 *T, Quat *Rq, M4 *S) {
    T->x = m.m[0][3]; T->y = m.m[1][3]; T->z = m.m[2][3];
    M4 M = m;
    for (int i = 0; i < 3; ++i) M.m[i][3] = M.m[3][i] = 0.f;
    M.m[3][3] = 1.f;
    float norm;
    int count = 0;
    M4 R = M;
    do {
        M4 Rnext;
        M4 Rit = Inverse(Transpose(R));
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) Rnext.m[i][j] = 0.5f * (R.m[i][j] + Rit.m[i][j]);
        norm = 0.f;
        for (int i = 0; i < 3; ++i) {
            float n = fabsf(R.m[i][0] - Rnext.m[i][0]) + fabsf(R.m[i][1] - Rnext.m[i][1]) +
                      fabsf(R.m[i][2] - Rnext.m[i][2]);
            norm = pmax(norm, n);
        }
        R = Rnext;
    } while (++count < 100 && norm > .0001f);
    *Rq = QuatFromXform(Xform(R));
    *S = Mul(Inverse(R), M);
}

AnimXform::AnimXform(const Xform &a, float t0, const Xform &b, float t1)
    : startTime(t0), endTime(t1), start(a), end(b), animated(a != b) {
    Decompose(start.m, &T[0], &R[0], &S[0]);
    Decompose(end.m, &T[1], &R[1], &S[1]);
}
// transform.cpp:356-381
void AnimXform::Interpolate(float time, Xform *t) const {
    if (!animated || time <= startTime) { *t = start; return; }
    if (time >= endTime) { *t = end; return; }
    float dt = (time - startTime) / (endTime - startTime);
    V3 trans = (1.f - dt) * T[0] + dt * T[1];
    Quat rotate = Slerp(dt, R[0], R[1]);
    M4 scale;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) scale.m[i][j] = Lerp(dt, S[0].m[i][j], S[1].m[i][j]);
    *t = Translate(trans) * QuatToXform(rotate) * Xform(scale);
}
BBox AnimXform::MotionBounds(const BBox &b, bool useInverse) const {
    if (!animated) return Inverse(start)(b);
    BBox ret;
    const int nSteps = 128;
    for (int i = 0; i < nSteps; ++i) {
        Xform t;
        float time = Lerp(float(i) / float(nSteps - 1), startTime, endTime);
        Interpolate(time, &t);
        if (useInverse) t = Inverse(t);
        ret = Union(ret, t(b));
    }
    return ret;
}

}  // namespace pbrtamd
