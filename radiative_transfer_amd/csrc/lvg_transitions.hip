// lvg_transitions.hip — post-processing of the level populations on gfx950:
// transition_data_container::find (transition_data.cpp:380-417) with calc_inv,
// calc_gain, calc_line_profile and calc_exc_temp (:210-377).
//
// Work: for every radiative line (u > l, A_ul > 0, the solver's plain line list)
// and every layer, the inversion, gain, excitation temperature and the line and
// dust opacities of the profile integral (tr_layer_kernel, one thread per (line,
// layer), coalesced along layers); the dz-weighted cloud averages in layer order
// (tr_reduce_kernel, one thread per line); for the inverted lines the optical depth
// over 37 aspect ratios x 300 velocities, each a sum over all layers of
// (kappa_line * exp(-x^2) - kappa_dust)^+ dz a (tr_profile_kernel, one thread per
// (line, velocity, aspect), sequential over layers as the reference sums), and the
// maxima over velocity (tr_aspect_kernel). Every floating-point operation follows
// the reference's expression order; exp/log come from include/lvg_math.h as in
// the solver, so the oracle (oracle_find_transitions) matches bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvg_device.h"
#include "../../include/lvg_amd.h"
#include "../../include/lvg_math.h"

namespace lvgtr {

constexpr double BOLTZMANN_CONSTANT    = 1.380649e-16;
constexpr double CM_INVERSE_TO_KELVINS = 1.438776877;
constexpr double EIGHT_PI              = 25.132741228718345;
constexpr double ONEDIVBY_SQRT_PI      = 0.56418958354775628;


// calc_inv / calc_gain / calc_line_profile per-layer parts / calc_exc_temp
__global__ void __launch_bounds__(256) tr_layer_kernel(const TrArgs *__restrict__ Ap) {
    const TrArgs &A = *Ap;
    const int lay = blockIdx.x * blockDim.x + threadIdx.x, n = blockIdx.y;
    if (lay >= A.nb_lay) return;
    const int N = A.N, u = A.line_u[n], l = A.line_l[n];
    const int64_t ld = A.soa_ld;
    const double T = A.soa[0 * ld + lay], mol = A.soa[7 * ld + lay], vt = A.soa[8 * ld + lay];
    const double up_pop = A.pops[(int64_t)lay * N + u], low_pop = A.pops[(int64_t)lay * N + l];
    const double gu = A.g[u], gl = A.g[l];
    const double inv = up_pop / gu - low_pop / gl;                       // :218
    const int64_t o = (int64_t)n * A.nb_lay + lay;
    A.inv[o] = inv;
    // find(): inv * g_u > rel_error * level_pop[u] of the FIRST layer (:398)
    if (inv * gu > A.rel_error * A.pops[u]) atomicOr(&A.inverted[n], 1);
    const double energy = A.line_e[n], energy_th = energy * energy * energy, aul = A.line_aul[n];
    double vel;
    if (u == A.h2o22_up && l == A.h2o22_low) {                           // :256-258
        const double a = sqrt(2. * BOLTZMANN_CONSTANT * T / A.mass) + 5.e+4;
        vel = sqrt(a * a + vt * vt);
    } else {
        vel = sqrt(2. * BOLTZMANN_CONSTANT * T / A.mass + vt * vt);       // :261-262
    }
    double d_abs = 0.;                                                   // dust_model::absorption
    for (int c = 0; c < A.nb_comp; c++) d_abs += A.line_sigma[(int64_t)c * A.nb_lines + n] * A.soa[(10 + c) * ld + lay];
    const double line_gain = inv * gu * aul * ONEDIVBY_SQRT_PI * mol / (energy_th * EIGHT_PI * vel);   // :266-268
    A.gain[o] = line_gain - d_abs;
    const double vwl = sqrt(2. * BOLTZMANN_CONSTANT * T / A.mass + vt * vt);   // :321-322
    A.lop[o] = inv * gu * aul * mol * ONEDIVBY_SQRT_PI / (energy_th * EIGHT_PI * vwl);   // :325-327
    A.dop[o] = d_abs;
    if (n == 0) A.vw[lay] = vwl;
    A.exc[o] = CM_INVERSE_TO_KELVINS * energy / lvg_log((low_pop * gu) / (up_pop * gl));   // :234-235
}

// the cloud averages of calc_inv / calc_gain, summed in layer order (one thread per line)
__global__ void __launch_bounds__(64) tr_reduce_kernel(const TrArgs *__restrict__ Ap) {
    const TrArgs &A = *Ap;
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= A.nb_lines) return;
    const double *iv = A.inv + (int64_t)n * A.nb_lay, *gn = A.gain + (int64_t)n * A.nb_lay;
    double inv = 0., gain = 0., tau_eff = 0., g = 0.;
    int hg = 0;
    for (int lay = 0; lay < A.nb_lay; lay++) {
        const double dz = A.dz[lay], ga = gn[lay];
        inv += iv[lay] * dz;
        gain += ga * dz;
        if (ga > 0.) tau_eff += ga * dz;
        if (ga > g) { g = ga; hg = lay; }
    }
    if (g < 1.e-99) hg = 0;
    A.line_sum[4 * n + 0] = inv / A.height;
    A.line_sum[4 * n + 1] = gain / A.height;
    A.line_sum[4 * n + 2] = tau_eff;
    A.line_sum[4 * n + 3] = (double)hg;
}

// calc_line_profile (:336-356): one thread per (selected line, velocity n, aspect i)
__global__ void __launch_bounds__(256) tr_profile_kernel(const TrArgs *__restrict__ Ap) {
    const TrArgs &A = *Ap;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = blockIdx.y;
    if (idx >= LVG_NB_FREQ * LVG_NB_ASPECT || k >= A.nb_sel) return;
    const int n = idx / LVG_NB_ASPECT, i = idx - n * LVG_NB_ASPECT;
    const int line = A.sel[k];
    const int L = A.nb_lay;
    const double vmax = A.vel_n[0] + A.velocity_shift, vmin = A.vel_n[L - 1] - A.velocity_shift;
    const double dv = (vmax - vmin) / (LVG_NB_FREQ - 1.);
    double vel = vmin;
    for (int q = 0; q < n; q++) vel += dv;                               // vel += dv per step (:339)
    const double aspect_ratio = 1. + A.delta_aspect * i;
    const double *lo = A.lop + (int64_t)line * L, *dp = A.dop + (int64_t)line * L;
    double acc = 0.;
    for (int lay = 0; lay < L; lay++) {
        const double x = (vel - A.vel_n[lay] / aspect_ratio) / A.vw[lay];
        const double profile = lvg_exp(-x * x);
        const double t = lo[lay] * profile - dp[lay];
        if (t > 0.) acc += t * A.dz[lay] * aspect_ratio;
    }
    A.od[((int64_t)k * LVG_NB_FREQ + n) * LVG_NB_ASPECT + i] = acc;
}

// maxima over velocity per aspect ratio (:359-366) and the aspect-1 spectrum (:370-372)
__global__ void __launch_bounds__(64) tr_aspect_kernel(const TrArgs *__restrict__ Ap) {
    const TrArgs &A = *Ap;
    const int k = blockIdx.x, t = threadIdx.x;
    if (k >= A.nb_sel) return;
    const double *od = A.od + (int64_t)k * LVG_NB_FREQ * LVG_NB_ASPECT;
    if (t < LVG_NB_ASPECT) {
        double x = 0.;
        for (int n = 0; n < LVG_NB_FREQ; n++)
            if (x < od[n * LVG_NB_ASPECT + t]) x = od[n * LVG_NB_ASPECT + t];
        A.tau_asp[k * LVG_NB_ASPECT + t] = x;
    }
    for (int n = t; n < LVG_NB_FREQ; n += blockDim.x) A.tau_freq[k * LVG_NB_FREQ + n] = od[n * LVG_NB_ASPECT];
}

}  // namespace lvgtr

extern "C" hipError_t lvg_tr_launch(int stage, const void *args_dev, int nb_lines, int nb_lay, int nb_sel,
                                    hipStream_t s) {
    const auto *A = static_cast<const lvgtr::TrArgs *>(args_dev);
    switch (stage) {
    case 0:
        hipLaunchKernelGGL(lvgtr::tr_layer_kernel, dim3((nb_lay + 255) / 256, nb_lines), dim3(256), 0, s, A);
        hipLaunchKernelGGL(lvgtr::tr_reduce_kernel, dim3((nb_lines + 63) / 64), dim3(64), 0, s, A);
        break;
    case 1:
        if (nb_sel > 0) {
            hipLaunchKernelGGL(lvgtr::tr_profile_kernel, dim3((LVG_NB_FREQ * LVG_NB_ASPECT + 255) / 256, nb_sel),
                               dim3(256), 0, s, A);
            hipLaunchKernelGGL(lvgtr::tr_aspect_kernel, dim3(nb_sel), dim3(64), 0, s, A);
        }
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

extern "C" size_t lvg_tr_args_size() { return sizeof(lvgtr::TrArgs); }
