// Control seeds and shape functions: restatement of the reference's
// SeedGenerator (include/SeedGenerator.hpp:12-126).  Same formulas, same
// (accumulating) grid construction, same use of rand() for the random seeds.
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <vector>

class SeedGenerator {
 public:
  // a, a+h, ... while <= b + 1e-7, h = (b-a)/(n-1), by repeated addition (:26-37)
  static std::vector<double> linspace(double a, double b, int n) {
    std::vector<double> grid;
    const double h = (b - a) / (n - 1);
    for (double x = a; x <= b + 1e-7; x += h) grid.push_back(x);
    return grid;
  }
  // MATLAB a:b:c by repeated addition (:39-48)
  static std::vector<double> generateRange(double a, double b, double c) {
    std::vector<double> grid;
    for (double x = a; x <= c + 1e-7; x += b) grid.push_back(x);
    return grid;
  }
  // 1 / (1 + exp(-k (x - offset))) elementwise (:50-58)
  static std::vector<double> sigmoid(std::vector<double>& x, double k, double offset) {
    std::vector<double> s(x.size());
    for (size_t i = 0; i < x.size(); ++i) s[i] = 1.0 / (1 + std::exp(-k * (x[i] - offset)));
    return s;
  }
  // randomised linear + sigmoid ramp with pinned endpoints (:66-95)
  static std::vector<double> linsigmoidSeed(double u_start, double u_end, size_t length) {
    std::vector<double> x = linspace(0, 100, int(length));
    const double a = randomDouble(0.01, 0.15);
    const double b = u_end - u_start - a * x.back();
    const double c = randomDouble(0.06, 0.18);
    const double d = randomDouble(60, 80);
    std::vector<double> shape = sigmoid(x, 0.7, 5), tail = sigmoid(x, -0.9, 100 - 7);
    for (size_t i = shape.size() / 2; i < shape.size(); ++i) shape[i] = tail[i];
    shape.front() = 0;
    shape.back() = 0;
    for (size_t i = 0; i < x.size(); ++i) {
      const double t = x[i];
      const double ramp = a * t + b / (1 + std::exp(-c * (t - d))) + u_start;
      const double base = (u_end - u_start) / (1 + std::exp(-0.2 * (t - 40))) + u_start;
      x[i] = shape[i] * ramp + (1 - shape[i]) * base;
    }
    return x;
  }
  // deterministic adiabatic-style ramp (:97-116)
  static std::vector<double> adiabaticSeed(double u_start, double u_end, size_t length) {
    std::vector<double> x = linspace(0, 100, int(length));
    const double p = 3.5, k = 1.0 / 3.0, xs = 40, a = 0.01;
    for (double& t : x) {
      if (t < xs) t = (p - u_start - a * xs) / (1 + std::exp(-k * (t - xs / 2.0))) + u_start + a * t;
      else t = std::exp(std::log(u_end - p + 1) / (100 - xs) * (t - xs)) + p - 1;
    }
    return x;
  }
  // N iid U(min, max) draws from rand() (:118-126)
  static std::vector<double> randomCoeffSeed(double min, double max, size_t N) {
    std::vector<double> v(N);
    for (double& x : v) x = randomDouble(min, max);
    return v;
  }

 private:
  static double randomDouble(double min, double max) {  // (:60-64)
    return min + (double)rand() / RAND_MAX * (max - min);
  }
};
