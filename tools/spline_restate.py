"""Independent restatement of the reference's track spline construction, in plain Python floats.

Written from the reference sources, not from oracle/ or the product's host_spline.cpp, so that the
product's host tables (mpcc_track_build_host / mpcc_track_eval_host) are checked against a second,
separately derived implementation (VERDICT r01 "clone against clone"):
  * CubicSpline::compSplineParams / getIndex / getPoint / getDerivative / getSecondDerivative
    (cpp/src/Spline/cubic_spline.cpp:65-246) — the natural cubic spline of the Wikipedia algorithm;
  * CubicSplineRot::compSplineRotParams / getPoint / getDerivative (cubic_spline_rot.cpp:142-259) with
    LogMatrix / ExpMatrix (:44-95, quirks Q10/Q11);
  * ArcLengthSpline::compArcLength / resamplePath / fitSpline / gen6DSpline (arc_length_spline.cpp:62-265):
    chord-length fit -> 100-point resample -> second fit -> resample -> regular final fit;
  * Eigen::VectorXd::LinSpaced(n, lo, hi) as used by resamplePath.
Python floats are IEEE doubles without FMA contraction; math.* are the C library's functions.
"""
import bisect
import math

N_SPLINE = 100  # config.h:38


def mat_mul(A, B):
    return [[A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j] for j in range(3)] for i in range(3)]


def transpose(A):
    return [[A[j][i] for j in range(3)] for i in range(3)]


def skew(v):
    return [[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]]


def inv_skew(S):
    return [S[2][1], S[0][2], S[1][0]]


def sym_eig(A):
    """Eigen-decomposition of the symmetric part read from the lower triangle (SelfAdjointEigenSolver),
    cyclic Jacobi; ascending eigenvalues, eigenvectors as columns.  Only LogMatrix's theta = pi branch."""
    M = [[A[max(i, j)][min(i, j)] for j in range(3)] for i in range(3)]
    V = [[1.0 if i == j else 0.0 for j in range(3)] for i in range(3)]
    for _ in range(60):
        off = abs(M[0][1]) + abs(M[0][2]) + abs(M[1][2])
        if off < 1e-300:
            break
        for p, q in ((0, 1), (0, 2), (1, 2)):
            if abs(M[p][q]) < 1e-300:
                continue
            th = (M[q][q] - M[p][p]) / (2 * M[p][q])
            t = (1.0 if th >= 0 else -1.0) / (abs(th) + math.sqrt(th * th + 1))
            c = 1 / math.sqrt(t * t + 1)
            s = t * c
            for k in range(3):
                mkp, mkq = M[k][p], M[k][q]
                M[k][p], M[k][q] = c * mkp - s * mkq, s * mkp + c * mkq
            for k in range(3):
                mpk, mqk = M[p][k], M[q][k]
                M[p][k], M[q][k] = c * mpk - s * mqk, s * mpk + c * mqk
            for k in range(3):
                vkp, vkq = V[k][p], V[k][q]
                V[k][p], V[k][q] = c * vkp - s * vkq, s * vkp + c * vkq
    order = sorted(range(3), key=lambda i: M[i][i])
    return [M[i][i] for i in order], [[V[r][i] for i in order] for r in range(3)]


def log_matrix(R):
    """LogMatrix (cubic_spline_rot.cpp:44-79)."""
    tr = R[0][0] + R[1][1] + R[2][2]
    if abs(tr + 1.0) < 1e-6:
        w, V = sym_eig(R)
        out = [[0.0] * 3 for _ in range(3)]
        for i in range(3):
            if abs(w[i] - 1.0) < 1e-4:
                u = [V[0][i], V[1][i], V[2][i]]
                n = math.sqrt(sum(x * x for x in u))
                S = skew([x / n for x in u])
                out = [[-S[a][b] * math.pi for b in range(3)] for a in range(3)]
        return out
    if abs(tr - 3.0) < 1e-6:
        return [[0.0] * 3 for _ in range(3)]
    th = math.acos((tr - 1.0) / 2.0)
    f = 1.0 / 2.0 * th / math.sin(th)
    return [[f * (R[a][b] - R[b][a]) for b in range(3)] for a in range(3)]


def exp_matrix(sk):
    """ExpMatrix (cubic_spline_rot.cpp:81-95); Q11: the small-angle branch's 1/2 is integer 0."""
    v = inv_skew(sk)
    vn = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    I = [[1.0 if a == b else 0.0 for b in range(3)] for a in range(3)]
    if vn <= 1e-8:
        return [[I[a][b] + math.cos(vn) * sk[a][b] for b in range(3)] for a in range(3)]
    sk2 = mat_mul(sk, sk)
    a1, b1 = math.sin(vn) / vn, (1 - math.cos(vn)) / (vn ** 2)
    return [[I[a][b] + a1 * sk[a][b] + b1 * sk2[a][b] for b in range(3)] for a in range(3)]


def lin_spaced(n, lo, hi):
    """Eigen LinSpaced (the linspaced_op of Eigen 3.4: from the far end when |hi| < |lo|)."""
    step = (hi - lo) / (n - 1)
    if abs(hi) < abs(lo):
        return [lo if i == 0 else hi - (n - 1 - i) * step for i in range(n)]
    return [hi if i == n - 1 else lo + i * step for i in range(n)]


class Spline1:
    """CubicSpline (cubic_spline.cpp:65-246)."""

    def __init__(self, x, y, regular):
        n = len(x)
        self.x, self.y, self.regular = list(x), list(y), regular
        self.dx = x[1] - x[0] if regular else 0.0
        a = list(y)
        h = [x[i + 1] - x[i] for i in range(n - 1)]
        alpha = [0.0] * (n - 1)
        for i in range(1, n - 1):
            alpha[i] = 3.0 / h[i] * (a[i + 1] - a[i]) - 3.0 / h[i - 1] * (a[i] - a[i - 1])
        l, mu, z = [0.0] * n, [0.0] * (n - 1), [0.0] * n
        l[0] = 1.0
        for i in range(1, n - 1):
            l[i] = 2.0 * (x[i + 1] - x[i - 1]) - h[i - 1] * mu[i - 1]
            mu[i] = h[i] / l[i]
            z[i] = (alpha[i] - h[i - 1] * z[i - 1]) / l[i]
        c = [0.0] * n
        b, d = [0.0] * (n - 1), [0.0] * (n - 1)
        for i in range(n - 2, -1, -1):
            c[i] = z[i] - mu[i] * c[i + 1]
            b[i] = (a[i + 1] - a[i]) / h[i] - (h[i] * (c[i + 1] + 2.0 * c[i])) / 3.0
            d[i] = (c[i + 1] - c[i]) / (3.0 * h[i])
        self.a, self.b, self.c, self.d = a, b, c, d
        # x_map: std::map<double, int> keeps the last index of equal keys
        self.keys = sorted({v: i for i, v in enumerate(x)}.items())

    def index(self, x):
        if x == self.x[-1]:
            return len(self.x) - 1
        if self.regular:
            return int(math.floor(x / self.dx))
        k = bisect.bisect_right([kv[0] for kv in self.keys], x)
        return -1 if k == len(self.keys) else self.keys[k][1] - 1

    def clamp(self, x):
        return max(0.0, min(x, self.x[-1]))

    def point(self, x):
        x = self.clamp(x)
        i = self.index(x)
        d1 = x - self.x[i]
        if i == len(self.x) - 1:
            return self.y[-1]
        return self.a[i] + self.b[i] * d1 + self.c[i] * (d1 * d1) + self.d[i] * (d1 * (d1 * d1))

    def deriv(self, x):
        x = self.clamp(x)
        i = self.index(x)
        d1 = x - self.x[i]
        if i == len(self.x) - 1:
            return 0.0
        return self.b[i] + 2.0 * self.c[i] * d1 + 3.0 * self.d[i] * (d1 * d1)

    def deriv2(self, x):
        x = self.clamp(x)
        i = self.index(x)
        d1 = x - self.x[i]
        if i == len(self.x) - 1:
            return 2.0 * self.c[i]
        return 2.0 * self.c[i] + 6.0 * self.d[i] * d1


class SplineRot(Spline1):
    """CubicSplineRot (cubic_spline_rot.cpp:142-259): c = 3/h^2, d = -2/h^3 on each interval."""

    def __init__(self, x, R, regular):
        n = len(x)
        self.x, self.R, self.regular = list(x), [list(map(list, r)) for r in R], regular
        self.dx = x[1] - x[0] if regular else 0.0
        self.c = [3.0 / math.pow(x[i + 1] - x[i], 2) for i in range(n - 1)]
        self.d = [-2.0 / math.pow(x[i + 1] - x[i], 3) for i in range(n - 1)]
        self.keys = sorted({v: i for i, v in enumerate(x)}.items())

    def point(self, x):
        x = self.clamp(x)
        i = self.index(x)
        if i == len(self.x) - 1:
            return self.R[-1]
        d1 = x - self.x[i]
        f = self.c[i] * (d1 * d1) + self.d[i] * (d1 * (d1 * d1))
        L = log_matrix(mat_mul(transpose(self.R[i]), self.R[i + 1]))
        return mat_mul(self.R[i], exp_matrix([[L[a][b] * f for b in range(3)] for a in range(3)]))

    def deriv(self, x):
        x = self.clamp(x)
        i = self.index(x)
        if i == len(self.x) - 1:
            return [0.0, 0.0, 0.0]
        d1 = x - self.x[i]
        v = inv_skew(log_matrix(mat_mul(transpose(self.R[i]), self.R[i + 1])))
        f = 2.0 * self.c[i] * d1 + 3.0 * self.d[i] * (d1 * d1)
        return [v[0] * f, v[1] * f, v[2] * f]


def arc_length(X, Y, Z):
    s = [0.0]
    for i in range(len(X) - 1):
        dx, dy, dz = X[i + 1] - X[i], Y[i + 1] - Y[i], Z[i + 1] - Z[i]
        s.append(s[-1] + math.sqrt(dx * dx + dy * dy + dz * dz))
    return s


def resample(fx, fy, fz, fr, total):
    s = lin_spaced(N_SPLINE, 0.0, total)
    return s, [fx.point(v) for v in s], [fy.point(v) for v in s], [fz.point(v) for v in s], [fr.point(v) for v in s]


def gen6d(X, Y, Z, R):
    """ArcLengthSpline::gen6DSpline (fitSpline, arc_length_spline.cpp:213-265).  Returns the final regular
    path data (s, X, Y, Z, R) and the four final splines."""
    s = arc_length(X, Y, Z)
    p1 = resample(Spline1(s, X, False), Spline1(s, Y, False), Spline1(s, Z, False), SplineRot(s, R, False), s[-1])
    s2 = arc_length(p1[1], p1[2], p1[3])
    p2 = resample(Spline1(s2, p1[1], False), Spline1(s2, p1[2], False), Spline1(s2, p1[3], False),
                  SplineRot(s2, p1[4], False), s2[-1])
    sf, Xf, Yf, Zf, Rf = p2
    fin = (Spline1(sf, Xf, True), Spline1(sf, Yf, True), Spline1(sf, Zf, True), SplineRot(sf, Rf, True))
    return (sf, Xf, Yf, Zf, Rf), fin


def evaluate(fin, s):
    """getPosition / getDerivative / getSecondDerivative / getOrientation / getOrientationDerivative."""
    fx, fy, fz, fr = fin
    return ([fx.point(s), fy.point(s), fz.point(s)], [fx.deriv(s), fy.deriv(s), fz.deriv(s)],
            [fx.deriv2(s), fy.deriv2(s), fz.deriv2(s)], fr.point(s), fr.deriv(s))
