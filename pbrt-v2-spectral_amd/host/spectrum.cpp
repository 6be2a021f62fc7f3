// spectrum.cpp -- host SampledSpectrum conversions (see spectrum.h for provenance).
#include "spectrum.h"
#include "pmath.h"
#include "spectral_tables.inc"
#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace pbrtamd {

// RGBSpectrum::y (spectrum.h:489-492): YWeight[0] c0 + YWeight[1] c1 + YWeight[2] c2, here as
// ((0 + w0 c0) + w1 c1) + w2 c2, divided by yint = 1 -- the same float result
static const float kRgbY[3] = {0.212671f, 0.715160f, 0.072169f};
static const float kRgbZero[3] = {0.f, 0.f, 0.f};

SpectrumCtx::SpectrumCtx(int nBands, int lambdaStart, int lambdaEnd) : nb(nBands), l0(lambdaStart), l1(lambdaEnd) {
    if (nBands == 3) {
        tX = kRgbZero; tY = kRgbY; tZ = kRgbZero; tyint = 1.f;
        for (int k = 0; k < 14; ++k) basis[k] = kRgbZero;   // FromRGB is the identity (no basis)
        return;
    }
    const SpectralTableSet *t = nullptr;
    if (nBands == 32 && l0 == 395 && l1 == 715) t = &kTables_32_395_715;
    else if (nBands == 60 && l0 == 395 && l1 == 715) t = &kTables_60_395_715;
    else if (nBands == 30 && l0 == 400 && l1 == 700) t = &kTables_30_400_700;
    if (!t) throw std::runtime_error("unsupported spectral band configuration");
    tX = t->X; tY = t->Y; tZ = t->Z; tyint = t->yint;
    for (int k = 0; k < 14; ++k) basis[k] = t->basis[k];
}

// r += a * B  (CoefficientSpectrum::operator*(float) then operator+=)
static inline void addScaled(Spec &r, float a, const float *B) {
    for (size_t i = 0; i < r.size(); ++i) r[i] += B[i] * a;
}

// spectrum.cpp:93-178 ; basis order: W C M Y R G B (reflectance 0-6, illuminant 7-13)
Spec SpectrumCtx::FromRGB(const float rgb[3], bool illum) const {
    if (this->rgb()) return Spec(rgb, rgb + 3);   // RGBSpectrum::FromRGB (spectrum.h:463-470): no clamp
    Spec r(nb, 0.f);
    const float *const *b = basis + (illum ? 7 : 0);
    enum { W, C, M, Yy, R, G, B };
    if (rgb[0] <= rgb[1] && rgb[0] <= rgb[2]) {
        addScaled(r, rgb[0], b[W]);
        if (rgb[1] <= rgb[2]) { addScaled(r, rgb[1] - rgb[0], b[C]); addScaled(r, rgb[2] - rgb[1], b[B]); }
        else { addScaled(r, rgb[2] - rgb[0], b[C]); addScaled(r, rgb[1] - rgb[2], b[G]); }
    } else if (rgb[1] <= rgb[0] && rgb[1] <= rgb[2]) {
        addScaled(r, rgb[1], b[W]);
        if (rgb[0] <= rgb[2]) { addScaled(r, rgb[0] - rgb[1], b[M]); addScaled(r, rgb[2] - rgb[0], b[B]); }
        else { addScaled(r, rgb[2] - rgb[1], b[M]); addScaled(r, rgb[0] - rgb[2], b[R]); }
    } else {
        addScaled(r, rgb[2], b[W]);
        if (rgb[0] <= rgb[1]) { addScaled(r, rgb[0] - rgb[2], b[Yy]); addScaled(r, rgb[1] - rgb[0], b[G]); }
        else { addScaled(r, rgb[1] - rgb[2], b[Yy]); addScaled(r, rgb[0] - rgb[1], b[R]); }
    }
    float s = illum ? .86445f : (float).94;
    for (auto &v : r) v *= s;
    return SpecClamp(r);
}

Spec SpectrumCtx::FromXYZ(const float xyz[3], bool illum) const {
    float rgb[3];   // spectrum.h:48-52 (RGBSpectrum::FromXYZ: XYZToRGB, no clamp)
    rgb[0] = 3.240479f * xyz[0] - 1.537150f * xyz[1] - 0.498535f * xyz[2];
    rgb[1] = -0.969256f * xyz[0] + 1.875991f * xyz[1] + 0.041556f * xyz[2];
    rgb[2] = 0.055648f * xyz[0] - 0.204043f * xyz[1] + 1.057311f * xyz[2];
    return FromRGB(rgb, illum);
}

// spectrum.cpp:199-212
static float InterpolateSpectrumSamples(const float *lambda, const float *vals, int n, float l) {
    if (l <= lambda[0]) return vals[0];
    if (l >= lambda[n - 1]) return vals[n - 1];
    for (int i = 0; i < n - 1; ++i)
        if (l >= lambda[i] && l <= lambda[i + 1]) return Lerp((l - lambda[i]) / (lambda[i + 1] - lambda[i]), vals[i], vals[i + 1]);
    throw std::runtime_error("InterpolateSpectrumSamples: unsorted wavelengths");
}

// SampledSpectrum::FromSampled (spectrum.h:276-295): band averages; the RGB build's
// RGBSpectrum::FromSampled (spectrum.h:493-516): XYZ by the 1 nm matching functions over the
// interpolated samples, each divided by sum(CIE_Y), then FromXYZ (XYZToRGB, no clamp)
Spec SpectrumCtx::FromSampled(const float *lambda, const float *v, int n) const {
    bool sorted = true;
    for (int i = 0; i < n - 1; ++i) if (lambda[i] > lambda[i + 1]) { sorted = false; break; }
    if (!sorted) {
        std::vector<std::pair<float, float> > sv;
        for (int i = 0; i < n; ++i) sv.push_back(std::make_pair(lambda[i], v[i]));
        std::sort(sv.begin(), sv.end());
        std::vector<float> sl(n), svv(n);
        for (int i = 0; i < n; ++i) { sl[i] = sv[i].first; svv[i] = sv[i].second; }
        return FromSampled(sl.data(), svv.data(), n);
    }
    if (rgb()) {
        float xyz[3] = {0.f, 0.f, 0.f}, yint = 0.f;
        for (int i = 0; i < kCIE_nsamples; ++i) {
            yint += kCIE_Y[i];
            const float val = InterpolateSpectrumSamples(lambda, v, n, (float)(kCIE_lambda_first + i));
            xyz[0] += val * kCIE_X[i];
            xyz[1] += val * kCIE_Y[i];
            xyz[2] += val * kCIE_Z[i];
        }
        for (int k = 0; k < 3; ++k) xyz[k] /= yint;
        return FromXYZ(xyz, false);
    }
    Spec r(nb, 0.f);
    for (int i = 0; i < nb; ++i) {
        float lambda0 = Lerp(float(i) / float(nb), (float)l0, (float)l1);
        float lambda1 = Lerp(float(i + 1) / float(nb), (float)l0, (float)l1);
        r[i] = AverageSpectrumSamples(lambda, v, n, lambda0, lambda1);
    }
    return r;
}

// spectrum.cpp:187-196 + paramset.cpp:116-131
Spec SpectrumCtx::Blackbody(float temp, float scale) const {
    const int n = kCIE_nsamples;
    std::vector<float> wl(n), vals(n);
    for (int i = 0; i < n; ++i) wl[i] = (float)(kCIE_lambda_first + i);
    if (temp <= 0) { for (int i = 0; i < n; ++i) vals[i] = 0.f; }
    else {
        const double C2 = 1.4388e7;
        double norm = pow(555.0, 5.0) * (exp(C2 / (555.0 * temp)) - 1.);
        for (int i = 0; i < n; ++i)
            vals[i] = float(norm / (pow(double(wl[i]), 5.0) * (exp(C2 / (wl[i] * temp)) - 1.)));
    }
    Spec s = FromSampled(wl.data(), vals.data(), n);
    for (auto &v : s) v *= scale;
    return s;
}

float SpectrumCtx::y(const Spec &s) const {
    float yy = 0.f;
    for (int i = 0; i < nb; ++i) yy += tY[i] * s[i];
    return yy / tyint;
}

void SpectrumCtx::ToRGB(const Spec &s, float rgb[3]) const {
    if (this->rgb()) { for (int k = 0; k < 3; ++k) rgb[k] = s[k]; return; }
    float xyz[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < nb; ++i) {
        xyz[0] += tX[i] * s[i];
        xyz[1] += tY[i] * s[i];
        xyz[2] += tZ[i] * s[i];
    }
    for (int k = 0; k < 3; ++k) xyz[k] /= tyint;
    rgb[0] = 3.240479f * xyz[0] - 1.537150f * xyz[1] - 0.498535f * xyz[2];
    rgb[1] = -0.969256f * xyz[0] + 1.875991f * xyz[1] + 0.041556f * xyz[2];
    rgb[2] = 0.055648f * xyz[0] - 0.204043f * xyz[1] + 1.057311f * xyz[2];
}

Spec SpecMul(const Spec &a, const Spec &b) {
    Spec r = a;
    for (size_t i = 0; i < r.size(); ++i) r[i] *= b[i];
    return r;
}
Spec SpecClamp(const Spec &a, float lo, float hi) {
    Spec r(a.size());
    for (size_t i = 0; i < a.size(); ++i) r[i] = Clamp(a[i], lo, hi);
    return r;
}
bool SpecIsBlack(const Spec &a) {
    for (float v : a) if (v != 0.) return false;
    return true;
}

// spectrum.cpp:50-83
float AverageSpectrumSamples(const float *lambda, const float *vals, int n, float lambdaStart, float lambdaEnd) {
    if (lambdaEnd <= lambda[0]) return vals[0];
    if (lambdaStart >= lambda[n - 1]) return vals[n - 1];
    if (n == 1) return vals[0];
    float sum = 0.f;
    if (lambdaStart < lambda[0]) sum += vals[0] * (lambda[0] - lambdaStart);
    if (lambdaEnd > lambda[n - 1]) sum += vals[n - 1] * (lambdaEnd - lambda[n - 1]);
    int i = 0;
    while (lambdaStart > lambda[i + 1]) ++i;
    for (; i + 1 < n && lambdaEnd >= lambda[i]; ++i) {
        float segStart = pmax(lambdaStart, lambda[i]);
        float segEnd = pmin(lambdaEnd, lambda[i + 1]);
        float a = Lerp((segStart - lambda[i]) / (lambda[i + 1] - lambda[i]), vals[i], vals[i + 1]);
        float b = Lerp((segEnd - lambda[i]) / (lambda[i + 1] - lambda[i]), vals[i], vals[i + 1]);
        sum += (0.5f * (a + b)) * (segEnd - segStart);
    }
    return sum / (lambdaEnd - lambdaStart);
}

}  // namespace pbrtamd
