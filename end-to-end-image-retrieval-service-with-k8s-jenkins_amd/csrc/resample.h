// resample.h — Pillow's resampling coefficients (host), shared by the embedding's
// device resize (vit.hip) and the fused JPEG decode → resize (jpeg.hip).
#pragma once

#include <cmath>
#include <stdexcept>
#include <vector>

#include "retrieval_core.h"

namespace rc {

// Restates libImaging/Resample.c precompute_coeffs + normalize_coeffs_8bpc
// (the same algorithm oracle/pil_resample.py pins against Pillow).
struct ResampleCoeffs {
    int ksize = 0;
    std::vector<int> bounds;  // [out][2] = (xmin, xcount)
    std::vector<int> coef;    // [out][ksize] fixed point, 22 fractional bits
};

inline double bicubic_filter(double x) {
    const double a = -0.5;
    if (x < 0.0) x = -x;
    if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1.0;
    if (x < 2.0) return (((x - 5.0) * x + 8.0) * x - 4.0) * a;
    return 0.0;
}
inline double bilinear_filter(double x) {
    if (x < 0.0) x = -x;
    if (x < 1.0) return 1.0 - x;
    return 0.0;
}

inline ResampleCoeffs precompute_coeffs(int in_size, int out_size, int resample) {
    double (*filt)(double) = resample == RC_RESAMPLE_BICUBIC ? bicubic_filter : bilinear_filter;
    const double fsupport = resample == RC_RESAMPLE_BICUBIC ? 2.0 : 1.0;
    const double in0 = 0.0, in1 = (double)in_size;
    const double scale = (in1 - in0) / out_size;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = fsupport * filterscale;
    ResampleCoeffs r;
    r.ksize = (int)std::ceil(support) * 2 + 1;
    r.bounds.assign(2 * out_size, 0);
    r.coef.assign((size_t)out_size * r.ksize, 0);
    std::vector<double> k(r.ksize);
    const double ss = 1.0 / filterscale;
    for (int xx = 0; xx < out_size; ++xx) {
        const double center = in0 + (xx + 0.5) * scale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        double ww = 0.0;
        for (int x = 0; x < xmax; ++x) {
            const double w = filt((x + xmin - center + 0.5) * ss);
            k[x] = w;
            ww += w;
        }
        for (int x = 0; x < xmax; ++x) {
            if (ww != 0.0) k[x] /= ww;
        }
        for (int x = 0; x < r.ksize; ++x) {
            const double v = x < xmax ? k[x] : 0.0;
            r.coef[(size_t)xx * r.ksize + x] = v < 0 ? (int)(-0.5 + v * (1 << 22)) : (int)(0.5 + v * (1 << 22));
            // the device taps multiply in 24 bits (resample_tap): |coef| < 2^23, i.e. |weight| < 2
            if (r.coef[(size_t)xx * r.ksize + x] >= (1 << 23) || r.coef[(size_t)xx * r.ksize + x] < -(1 << 23))
                throw std::runtime_error("resample weight out of the 24-bit tap range");
        }
        r.bounds[2 * xx] = xmin;
        r.bounds[2 * xx + 1] = xmax;
    }
    return r;
}

}  // namespace rc
