// hq_host.cpp -- host-only parts of libhq: S-CIELAB filter design and the SWASA
// policy + findBestQuantization driver.  Compiled with -ffp-contract=off so
// every float expression rounds like the Java original (no fused multiply-add).
//
// References (src/plugins/dbrasseur/hybridquantization/):
//   SP = ScielabProcessor.java (filter design SP:66-254),
//   IM = ImageManipulation.java (packing IM:800-841, driver IM:383-591),
//   SW = SWASA.java (policy SW:3-116).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "hq_swasa.h"

namespace {

// SP:44-53
const float kWeights[3][3] = {{1.00327f, 0.114416f, -0.117686f}, {0.616725f, 0.383275f, 0.f},
                              {0.567885f, 0.432115f, 0.f}};
const float kHalfwidths[3][3] = {{0.05f, 0.225f, 7.0f}, {0.0685f, 0.826f, 0.f},
                                 {0.0920f, 0.6451f, 0.f}};
const int kNumFilters[3] = {3, 2, 2};
const float kD65[3] = {0.95047f, 1.0f, 1.0883f};   // SP:20
const float kD50[3] = {0.966797f, 1.0f, 0.825188f};  // SP:21
const int kMinSampPerDeg = 224;                      // SP:23

// SP:238-254 gauss(halfwidth, width): Java float/double promotion kept.
std::vector<float> gauss(float halfwidth, int width) {
    const float alpha = (2.0f * (float)std::sqrt(std::log(2.0))) / (halfwidth - 1.0f);
    std::vector<float> res(width);
    const int offset = width / 2;
    double sum = 0.0;
    for (int i = 0; i < width; ++i) {
        const float d = (float)(i - offset);
        const float e = ((-alpha * alpha) * d) * d;
        res[i] = (float)std::exp((double)e);
        sum += res[i];
    }
    for (int i = 0; i < width; ++i) res[i] = (float)((double)res[i] / sum);
    return res;
}

// SP:185-201 conv1D(data, filter): zero outside, float multiply then add.
std::vector<float> conv1d(const std::vector<float>& data, const std::vector<float>& filter) {
    const int n = (int)data.size();
    const int off = (int)filter.size() / 2;
    std::vector<float> res(n, 0.0f);
    for (int i = 0; i < n; ++i)
        for (int j = -off; j <= off; ++j)
            if (!(i + j < 0 || i + j >= n)) {
                const float prod = filter[j + off] * data[i + j];
                res[i] = res[i] + prod;
            }
    return res;
}

// SP:203-220
std::vector<float> resize1d(const std::vector<float>& src, int new_size) {
    std::vector<float> res(new_size, 0.0f);
    const int pad = std::abs(new_size - (int)src.size()) / 2;
    if (new_size > (int)src.size()) {
        for (size_t j = 0; j < src.size(); ++j) res[pad + j] = src[j];
    } else {
        for (int i = 0; i < new_size; ++i) res[i] = src[pad + i];
    }
    return res;
}

}  // namespace

extern "C" int hq_design_filters(int dpi, double viewing_distance, int whitepoint, int max_taps,
                                 float* k1, float* k2, float* k3, float* absk3, int* taps,
                                 float* illum) {
    if (dpi <= 0 || !(viewing_distance > 0) || !k1 || !k2 || !k3 || !absk3 || !taps)
        return HQ_ERR_ARG;
    // SP:79-88
    int spd = (int)std::floor(dpi / ((180 / M_PI) * std::atan(2.54 / viewing_distance)) + 0.5);
    if (spd <= 0) return HQ_ERR_ARG;
    int uprate;
    if (spd < kMinSampPerDeg) {
        uprate = (int)std::ceil(kMinSampPerDeg * 1.0 / spd);
        spd *= uprate;
    } else {
        uprate = 1;
    }
    // SP:91-99, SP:102
    float spreads[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < kNumFilters[i]; ++j) spreads[i][j] = kHalfwidths[i][j] * (float)spd;
    const int width = (int)std::ceil(spd / 2.0) * 2 - 1;
    // SP:104-119
    std::vector<float> of[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < kNumFilters[i]; ++j) {
            of[i][j] = gauss(spreads[i][j], width);
            const float w = kWeights[i][j];
            const float sgn = w > 0 ? 1.0f : (w < 0 ? -1.0f : 0.0f);
            const float factor = (float)std::sqrt((double)std::fabs(w)) * sgn;
            for (float& v : of[i][j]) v *= factor;
        }
    // SP:122-173
    if (uprate > 1) {
        std::vector<float> upcol(uprate * 2 - 1);
        for (int i = 0; i < (int)upcol.size(); ++i)
            upcol[i] = ((float)(uprate - std::abs(uprate - i - 1)) * 1.0f) / (float)uprate;
        upcol = resize1d(upcol, (int)upcol.size() + width - 1);
        std::vector<float> ups[3][3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < kNumFilters[i]; ++j) ups[i][j] = conv1d(of[i][j], upcol);
        const int s = (int)ups[0][0].size();
        const int mid = s / 2;
        const int nd = 2 * (mid / uprate) + 1;
        std::vector<int> temp;
        for (int v = mid, c = 0; c < (mid / uprate) + 1; v -= uprate, ++c) temp.push_back(v);
        std::reverse(temp.begin(), temp.end());
        std::vector<int> downs(nd);
        for (int i = 0, j = mid + uprate; i < nd; ++i) {
            if ((int)temp.size() > i) downs[i] = temp[i];
            else { downs[i] = j; j += uprate; }
        }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < kNumFilters[i]; ++j) {
                std::vector<float> r(nd);
                for (int t = 0; t < nd; ++t) r[t] = ups[i][j][downs[t]];
                of[i][j] = r;
            }
    }
    const int T = (int)of[0][0].size();
    *taps = T;
    if (T > max_taps) return HQ_ERR_UNSUPPORTED;
    // IM:800-841 packing + SP:174-178 abs filter
    for (int t = 0; t < T; ++t) {
        for (int c = 0; c < 3; ++c) {
            k1[4 * t + c] = of[c][0][t];
            k2[4 * t + c] = of[c][1][t];
        }
        k1[4 * t + 3] = 0.0f;
        k2[4 * t + 3] = 0.0f;
        k3[t] = of[0][2][t];
        absk3[t] = of[0][2][t] * (of[0][2][t] < 0 ? -1.0f : 1.0f);
    }
    if (illum) std::memcpy(illum, whitepoint == HQ_WP_D50 ? kD50 : kD65, sizeof(kD65));
    return HQ_OK;
}

extern "C" void hq_swasa_default_params(hq_swasa_params* p) {
    // HQ:192-224 GUI defaults
    p->population = 4;
    p->imax = 5000;
    p->iTc = 20;
    p->delta = 2.0f;
    p->conv_delay = 0.75f;
    p->conv_spread = 0.15f;
    p->t0 = 20.0f;
    p->alpha = 0.9f;
    p->s0 = 100.0f;
    p->beta = 5.3f;
    p->convergence = 1;
}

namespace hq {

Swasa::Swasa(const hq_swasa_params& p, uint64_t seed) : p_(p), rng_(seed) { reset(); }

void Swasa::reset() {
    temperature_ = p_.t0;
    step_width_ = p_.s0;
}

void Swasa::generate_random_colors(int K, float* out) {
    for (int i = 0; i < K; ++i) {
        out[4 * i + 0] = rng_.next_float();
        out[4 * i + 1] = rng_.next_float();
        out[4 * i + 2] = rng_.next_float();
        out[4 * i + 3] = 0.0f;
    }
}

bool Swasa::is_accepted(double delta_e) {
    // short-circuit: no random number is drawn when delta_e <= 0 (SW:56)
    return delta_e <= 0 || std::exp(-delta_e / (double)temperature_) > rng_.next_double();
}

double Swasa::keep_threshold(int iteration) const {
    const float num = (float)iteration - p_.conv_delay * (float)p_.imax;
    const float den = p_.conv_spread * (float)p_.imax;
    return -(std::tanh((double)(num / den))) / 2 + 0.5;
}

bool Swasa::keeps_his_values(int iteration) {
    return keep_threshold(iteration) > rng_.next_double();
}

float Swasa::max_step_width(int i) const {
    const float e = (p_.beta * (float)i) / (float)p_.imax;
    return (float)((double)(2.0f * p_.s0) / (1 + std::exp((double)e)));
}

double Swasa::compute_penalty(const int32_t* used, int K) const {
    double penalty = 0;
    for (int k = 0; k < K; ++k)
        if (used[k] == 0) penalty += p_.delta;
    return penalty;
}

void Swasa::reduce_temperature_if_necessary(int iteration) {
    if (iteration % p_.iTc == 0) temperature_ *= p_.alpha;
}

static inline float clampf_java(float v, float lo, float hi) {  // SW:103-106
    return v > lo ? (v > hi ? hi : v) : lo;
}

void Swasa::generate_neighboring_colors(const float* colors, float* next, int K, int iteration) {
    const float amax = max_step_width(iteration) / 256.0f;
    for (int i = 0; i < K; ++i) {
        const int o = 4 * i;
        for (int c = 0; c < 3; ++c) {
            const float u = rng_.next_float();
            const float step = (u * 2 - 1) * amax;
            next[o + c] = clampf_java(colors[o + c] + step, 0, 1);
        }
        next[o + 3] = 0.0f;
    }
}

SearchDriver::SearchDriver(const hq_swasa_params& p, int K, uint64_t seed, PopulationEval eval)
    : sw_(p, seed), K_(K), P_(p.population), eval_(std::move(eval)) {}

static int argmin_first(const std::vector<double>& a) {  // IM:843-856
    int m = 0;
    double s = a[0];
    for (size_t i = 1; i < a.size(); ++i)
        if (s > a[i]) { m = (int)i; s = a[i]; }
    return m;
}

int SearchDriver::start() {
    const int n = 4 * K_;
    sw_.reset();                                                   // IM:385
    colors_.assign((size_t)P_ * n, 0.0f);
    current_.assign((size_t)P_ * n, 0.0f);
    for (int i = 0; i < P_; ++i) sw_.generate_random_colors(K_, &colors_[(size_t)i * n]);  // IM:413-417
    current_errors_.assign(P_, 0.0);
    errors_.assign(P_, 0.0);
    int rc = eval_(colors_.data(), P_, K_, current_errors_.data());  // IM:490
    if (rc) return rc;
    const int m = argmin_first(current_errors_);                     // IM:491-493
    best_error_ = current_errors_[m];
    best_colors_.assign(colors_.begin() + (size_t)m * n, colors_.begin() + (size_t)(m + 1) * n);
    ite_ = 0;
    started_ = true;
    return HQ_OK;
}

int SearchDriver::run(int iterations, int* ran, std::vector<double>* trace) {
    if (!started_) return HQ_ERR_STATE;
    const int n = 4 * K_;
    const hq_swasa_params& p = sw_.params();
    int done = 0;
    for (; done < iterations && ite_ < p.imax; ++done) {
        const int ite = ++ite_;                                       // IM:497
        sw_.reduce_temperature_if_necessary(ite);                     // IM:507
        for (int j = 0; j < P_; ++j)                                  // IM:508-511
            sw_.generate_neighboring_colors(&colors_[(size_t)j * n], &current_[(size_t)j * n], K_, ite);
        int rc = eval_(current_.data(), P_, K_, errors_.data());      // IM:515
        if (rc) { if (ran) *ran = done; return rc; }
        double minerror = std::numeric_limits<double>::max();
        int minidx = 0;
        for (int i = 0; i < P_; ++i) {                                // IM:518-537
            if (P_ > 1 && errors_[i] < minerror) { minerror = errors_[i]; minidx = i; }
            if (sw_.is_accepted(errors_[i] - current_errors_[i])) {
                current_errors_[i] = errors_[i];
                std::copy_n(&current_[(size_t)i * n], n, &colors_[(size_t)i * n]);
                if (current_errors_[i] < best_error_) {
                    best_error_ = current_errors_[i];
                    std::copy_n(&current_[(size_t)i * n], n, best_colors_.data());
                }
            }
        }
        for (int i = 0; p.convergence && P_ > 1 && i < P_; ++i) {     // IM:538-545
            if (!sw_.keeps_his_values(ite)) {
                current_errors_[i] = minerror;
                std::copy_n(&current_[(size_t)minidx * n], n, &colors_[(size_t)i * n]);
            }
        }
        if (trace) {
            trace->push_back(best_error_);
            for (int i = 0; i < P_; ++i) trace->push_back(errors_[i]);
        }
    }
    if (ran) *ran = done;
    return HQ_OK;
}

}  // namespace hq

extern "C" int hq_swasa_search_host(const hq_swasa_params* params, int K, uint64_t seed,
                                    int iterations, hq_eval_fn eval, void* user,
                                    float* best_colors, double* best_error, double* trace) {
    if (!params || !eval || K < 1 || params->population < 1 || params->imax < 1 ||
        params->iTc < 1)
        return HQ_ERR_ARG;
    hq::SearchDriver d(*params, K, seed, [&](const float* pal, int P, int KK, double* costs) {
        return eval(user, pal, P, KK, costs) ? HQ_ERR_ARG : HQ_OK;
    });
    int rc = d.start();
    if (rc) return rc;
    std::vector<double> tr;
    int ran = 0;
    rc = d.run(iterations, &ran, trace ? &tr : nullptr);
    if (rc) return rc;
    if (best_colors) std::copy(d.best_colors().begin(), d.best_colors().end(), best_colors);
    if (best_error) *best_error = d.best_error();
    if (trace) std::copy(tr.begin(), tr.end(), trace);
    return HQ_OK;
}
