"""Integrator of the kinematic model (cpp/src/Model/integrator.cpp:29-68, model.cpp:31-45), vectorized
over instances on the host.  Used to drive closed loops (the caller of the hot path, main.cpp:100-114)."""
import numpy as np


def _f(x, u):
    f = np.empty_like(x)
    f[..., :7] = u[..., :7]
    f[..., 7] = x[..., 8]
    f[..., 8] = u[..., 7]
    return f


def rk4(x, u, ts):
    """Integrator::RK4 (integrator.cpp:29-43)."""
    x = np.asarray(x, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    k1 = _f(x, u)
    k2 = _f(x + ts / 2. * k1, u)
    k3 = _f(x + ts / 2. * k2, u)
    k4 = _f(x + ts * k3, u)
    return x + ts * (k1 / 6. + k2 / 3. + k3 / 3. + k4 / 6.)


def sim_time_step(x, u, ts, fine_time_step=0.001):
    """Integrator::simTimeStep (integrator.cpp:55-68): ts/1ms RK4 sub-steps."""
    steps = int(ts / fine_time_step)
    for _ in range(steps):
        x = rk4(x, u, fine_time_step)
    return x
