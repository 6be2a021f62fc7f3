// spectrum.h -- host-side SampledSpectrum with a run-time band count (32 or 60 in the
// configs).  Restates core/spectrum.{h,cpp}: FromRGB (spectrum.cpp:93-178),
// FromSampled / AverageSpectrumSamples (spectrum.h:277-296, spectrum.cpp:50-83) and
// the band tables of SampledSpectrum::Init (generated into spectral_tables.inc).
#pragma once
#include <vector>
#include <string>
#include <cmath>

namespace pbrtamd {

struct SpectralTables;   // opaque, see spectrum.cpp

class SpectrumCtx {
public:
    // n = 32 (395-715 nm, the reference build), 60 (395-715) or 30 (400-700); n = 3 is the
    // reference's RGB build (Spectrum = RGBSpectrum, pbrt.h:144; spectrum.h:453-530): FromRGB
    // keeps the triple, y() weighs it with YWeight (yint 1)
    explicit SpectrumCtx(int nBands, int lambdaStart = 395, int lambdaEnd = 715);
    int n() const { return nb; }
    bool rgb() const { return nb == 3; }
    int lambdaStart() const { return l0; }
    int lambdaEnd() const { return l1; }
    typedef std::vector<float> Spec;
    Spec Const(float v) const { return Spec(nb, v); }
    Spec FromRGB(const float rgb[3], bool illuminant = false) const;
    Spec FromXYZ(const float xyz[3], bool illuminant = false) const;
    Spec FromSampled(const float *lambda, const float *v, int n) const;
    Spec Blackbody(float tempK, float scale) const;
    float y(const Spec &s) const;
    // SampledSpectrum::ToRGB (spectrum.h:352-362, 423-427): ToXYZ then XYZToRGB
    void ToRGB(const Spec &s, float rgb[3]) const;
    const float *Basis(int k) const { return basis[k]; }   // FromRGB basis, order as in FromRGB
    const float *Y() const { return tY; }
    float yint() const { return tyint; }
private:
    int nb, l0, l1;
    const float *tX, *tY, *tZ;
    float tyint;
    const float *basis[14];
};

typedef std::vector<float> Spec;
Spec SpecMul(const Spec &a, const Spec &b);
Spec SpecClamp(const Spec &a, float lo = 0.f, float hi = INFINITY);
bool SpecIsBlack(const Spec &a);

float AverageSpectrumSamples(const float *lambda, const float *vals, int n, float l0, float l1);

}  // namespace pbrtamd
