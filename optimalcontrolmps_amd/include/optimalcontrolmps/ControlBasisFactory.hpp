// Chopped-sine GROUP basis: restatement of the reference's
// ControlBasisFactory::buildChoppedSineBasis (include/ControlBasisFactory.hpp:25-53).
//   shape S = sigmoid(x, 8, 1.1) on the first half, sigmoid(x, -8, 98.9) on
//   the second (x = linspace(0, 100, N)), with S_0 = S_{N-1} = 0;
//   f_{i n} = sin((n+1) PI tstep i / T) with the reference's PI = 3.14159265.
#pragma once

#include <cassert>
#include <cmath>
#include <vector>

#include "ControlBasis.hpp"
#include "SeedGenerator.hpp"

class ControlBasisFactory {
 public:
  static constexpr double kPi = 3.14159265;  // reference #define PI (include/ControlBasisFactory.hpp:9)

  static ControlBasis buildChoppedSineBasis(ocmps::stdvec& u0, double tstep, double T, size_t M) {
    const size_t N = u0.size();
    assert(N - (1 + T / tstep) < 1e-5);
    std::vector<double> x = SeedGenerator::linspace(0, 100, int(N));
    std::vector<double> rise = SeedGenerator::sigmoid(x, 8.0, 1.1);
    std::vector<double> fall = SeedGenerator::sigmoid(x, -8.0, 100 - 1.1);
    std::vector<double> S(N);
    for (size_t i = 0; i < N; ++i) S[i] = (i < N / 2) ? rise[i] : fall[i];
    S[0] = 0;
    S[N - 1] = 0;
    ocmps::rowmat f(N, std::vector<double>(M, 0.0));
    for (size_t i = 0; i < N; ++i)
      for (size_t n = 0; n < M; ++n) f[i][n] = std::sin((n + 1) * kPi * tstep * i / T);
    return ControlBasis(u0, S, f);
  }
};
