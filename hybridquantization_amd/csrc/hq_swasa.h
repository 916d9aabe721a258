// hq_swasa.h -- host-side SWASA policy and search driver (internal).
//
// SW:3-116 (policy) and IM:383-591 (findBestQuantization main loop) restated
// in C++.  The population evaluator is abstract so the same driver runs on the
// GPU context (hq_search_*) and on a host callback (hq_swasa_search_host).
#pragma once

#include <cmath>
#include <cstdint>
#include <functional>
#include <vector>

#include "../../include/hq.h"

namespace hq {

// java.util.Random: 48-bit LCG; nextFloat = next(24)/2^24; nextDouble 53 bits.
class JavaRandom {
   public:
    explicit JavaRandom(uint64_t seed) { set_seed(seed); }
    void set_seed(uint64_t s) { seed_ = (s ^ kMult) & kMask; }
    int32_t next(int bits) {
        seed_ = (seed_ * kMult + 0xBull) & kMask;
        return (int32_t)(int64_t)(seed_ >> (48 - bits));
    }
    float next_float() { return (float)next(24) / (float)(1 << 24); }
    double next_double() {
        return (double)(((int64_t)next(26) << 27) + next(27)) * (1.0 / (double)(1LL << 53));
    }

   private:
    static constexpr uint64_t kMult = 0x5DEECE66Dull;
    static constexpr uint64_t kMask = (1ull << 48) - 1;
    uint64_t seed_;
};

// SW:3-116.  Fields kept in fp32 like the Java class.
class Swasa {
   public:
    Swasa(const hq_swasa_params& p, uint64_t seed);
    void reset();                                           // SW:30-34
    void generate_random_colors(int K, float* out) ;        // SW:40-52
    bool is_accepted(double delta_e);                       // SW:54-57
    bool keeps_his_values(int iteration);                   // SW:59-62
    double keep_threshold(int iteration) const;             // its left-hand side
    float max_step_width(int i) const;                      // SW:69-72
    double compute_penalty(const int32_t* used, int K) const;  // SW:74-82
    void reduce_temperature_if_necessary(int iteration);    // SW:84-89
    void generate_neighboring_colors(const float* colors, float* next, int K, int iteration);  // SW:91-101
    const hq_swasa_params& params() const { return p_; }
    float temperature() const { return temperature_; }

   private:
    hq_swasa_params p_;
    JavaRandom rng_;
    float temperature_, step_width_;
};

using PopulationEval = std::function<int(const float* palettes, int P, int K, double* costs)>;

// IM:383-591 as a resumable state machine.
class SearchDriver {
   public:
    SearchDriver(const hq_swasa_params& p, int K, uint64_t seed, PopulationEval eval);
    int start();                          // IM:385-493: reset, initial population, argmin
    int run(int iterations, int* ran, std::vector<double>* trace);   // IM:497-568
    const std::vector<float>& best_colors() const { return best_colors_; }
    double best_error() const { return best_error_; }
    int iteration() const { return ite_; }

   private:
    Swasa sw_;
    int K_, P_;
    PopulationEval eval_;
    std::vector<float> colors_, current_;   // [P][4K]
    std::vector<double> current_errors_, errors_;
    std::vector<float> best_colors_;
    double best_error_ = 0.0;
    int ite_ = 0;
    bool started_ = false;
};

}  // namespace hq
