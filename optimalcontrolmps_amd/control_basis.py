"""GROUP control parameterisation on the host (Python mirror of the C++ facade's
ControlBasis / ControlBasisFactory / SeedGenerator, which restate the
reference's include/ControlBasis.hpp:13-37, src/ControlBasis.cpp:49-124,
include/ControlBasisFactory.hpp:25-53 and include/SeedGenerator.hpp:26-116).

Same formulas and the same accumulation order as the C++ restatement, so u,
the control Jacobian and the projected Hessian agree with it bit for bit; the
Hessian projection V H_u V^T itself runs on the device (ocg_convert_hessian,
Engine.convert_hessian) in the reference's inner-product order.
"""
from __future__ import annotations

import math

import numpy as np

PI = 3.14159265  # the reference's #define PI (include/ControlBasisFactory.hpp:9)


def linspace(a, b, n):
    """a, a+h, ... while <= b + 1e-7, h = (b-a)/(n-1), by repeated addition (SeedGenerator.hpp:26-37)"""
    h = (b - a) / (n - 1)
    out, x = [], a
    while x <= b + 1e-7:
        out.append(x)
        x += h
    return out


def sigmoid(x, k, offset):
    """1 / (1 + exp(-k (x - offset))) elementwise (SeedGenerator.hpp:50-58)"""
    return [1.0 / (1 + math.exp(-k * (t - offset))) for t in x]


def adiabatic_seed(u_start, u_end, length):
    """deterministic adiabatic-style ramp (SeedGenerator.hpp:97-116)"""
    p, k, xs, a = 3.5, 1.0 / 3.0, 40.0, 0.01
    out = []
    for t in linspace(0, 100, length):
        if t < xs:
            out.append((p - u_start - a * xs) / (1 + math.exp(-k * (t - xs / 2.0))) + u_start + a * t)
        else:
            out.append(math.exp(math.log(u_end - p + 1) / (100 - xs) * (t - xs)) + p - 1)
    return out


class ControlBasis:
    """u = u0 + S * (f c) (convertControl); V[n][i] = S_i f_{i n} (the transposed
    control Jacobian, the operand of convertHessian H_c = V H_u V^T)."""

    def __init__(self, u0, S, f):
        self.u0 = [float(x) for x in u0]
        self.S = [float(x) for x in S]
        self.f = [[float(x) for x in row] for row in f]
        self.N = len(self.u0)
        self.M = len(self.f[0]) if self.f else 0
        self.V = np.array([[self.f[i][n] * self.S[i] for i in range(self.N)] for n in range(self.M)])
        self.ucurrent = list(self.u0)

    def convert_control(self, c, new_control=True):
        """src/ControlBasis.cpp:49-66 (new_control == False: the cached u)"""
        if not new_control:
            return np.array(self.ucurrent)
        assert len(c) == self.M
        u = list(self.u0)
        for i in range(self.N):
            fc = 0.0
            for n in range(self.M):
                fc += self.f[i][n] * float(c[n])
            u[i] += self.S[i] * fc
        self.ucurrent = u
        return np.array(u)

    def convert_gradient(self, gu):
        """src/ControlBasis.cpp:69-88"""
        out = []
        for n in range(self.M):
            acc = 0.0
            for i in range(self.N):
                acc += self.S[i] * float(gu[i]) * self.f[i][n]
            out.append(acc)
        return np.array(out)

    def control_jacobian(self):
        return self.V.T.copy()


def build_chopped_sine_basis(u0, tstep, T, M):
    """ControlBasisFactory::buildChoppedSineBasis (include/ControlBasisFactory.hpp:25-53)"""
    N = len(u0)
    assert N - (1 + T / tstep) < 1e-5
    x = linspace(0, 100, N)
    rise, fall = sigmoid(x, 8.0, 1.1), sigmoid(x, -8.0, 100 - 1.1)
    S = [rise[i] if i < N // 2 else fall[i] for i in range(N)]
    S[0] = 0.0
    S[N - 1] = 0.0
    f = [[math.sin((n + 1) * PI * tstep * i / T) for n in range(M)] for i in range(N)]
    return ControlBasis(u0, S, f)


def regularization_hessian(n, gamma, tstep):
    """calcRegularizationHessian (src/OptimalControl.cpp:124-143): tridiagonal
    gamma/dt stencil, edges zero, H[1][0] = H[N-2][N-1] = 0"""
    H = np.zeros((n, n))
    g = gamma / tstep
    for i in range(1, n - 1):
        H[i, i - 1] = -g
        H[i, i + 1] = -g
        H[i, i] = 2 * g
    H[1, 0] = 0.0
    H[n - 2, n - 1] = 0.0
    return H
