"""Independent restatement of the per-stage robot record (RobotData, cpp/include/Model/robot_data.h:55-88) in numpy:
Panda kinematics, manipulability and both collision networks, written from the reference sources, not from oracle/
or the product (VERDICT r03 "What's missing" 1, next-round item 4).

  * RobotModel::setPanda (cpp/src/Model/robot_model.cpp:68-319): the joint frames as RBDL builds them, each body
    added with SpatialTransform(E, r) (E the rotation from the parent's to the body's coordinates, r the joint's
    position in the parent's coordinates) and, for the 7 arm joints, a revolute joint about the body's z axis, whose
    RBDL transform is Xrotz(q) (E_J = Rz(q)^T) applied after the fixed one: so a body's world orientation is
    R_parent E^T Rz(q) and its origin p_parent + R_parent r (the hand and its tcp frame are fixed, quirk Q19: the
    literal 0.707107 of the hand rotation);
  * getEEPosition / getEEOrientation (CalcBodyToBaseCoordinates, CalcBodyWorldOrientation^T) and getJacobian
    (CalcPointJacobian6D at the tcp origin, rows reordered to [Jv; Jw], robot_model.cpp:366-398): for a revolute
    joint j with world axis z_j through p_j, Jw_j = z_j, Jv_j = z_j x (p_tcp - p_j);
  * Manipulability sqrt(det(J J^T)) and its central difference with delta 1e-4 (robot_model.cpp:431-450);
  * SelCollNNmodel / EnvCollNNmodel::calculateMlpOutput (SelfCollisionModel.cpp:140-250, EnvCollisionModel.cpp:
    137-247): NeRF input [x, sin x, cos x], ReLU layers (ReLU'(0) = 0), value and the chain-rule Jacobian
    W_L D_{L-1} W_{L-1} ... D_0 W_0 J_nerf, sizes from osqp_interface.cpp:35-43 (self 7 -> 256 -> 64 -> 1, env
    10 -> 256 x 4 -> 9), weights read from the reference's own parameter text files (cpp/NNmodel/*/parameter);
  * RobotData::update / updateEnv: the env network sees [q, obstacle xyz] and only its 9 x 7 joint block is kept
    (robot_data.h:85, Q17).
The record layout is tools/qp_restate.py's REC_* (the fixture layout).  Test infrastructure only.
"""
import math
import os

import numpy as np

DOF, NLINK = 7, 9
# cpp/src/Model/robot_model.cpp:176-184 (joint_position) and :188-249 (joint_rotation = E), bodies 1..7, hand, tcp
JOINT_POS = [(0.0, 0.0, 0.333), (0.0, 0.0, 0.0), (0.0, -0.316, 0.0), (0.0825, 0.0, 0.0), (-0.0825, 0.384, 0.0),
             (0.0, 0.0, 0.0), (0.088, 0.0, 0.0)]
E_X = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, -1.0], [0.0, 1.0, 0.0]])    # links 2, 5
E_XN = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 1.0], [0.0, -1.0, 0.0]])   # links 3, 4, 6, 7
JOINT_ROT = [np.eye(3), E_X, E_XN, E_XN, E_X, E_XN, E_XN]
HAND_POS, HAND_ROT = (0.0, 0.0, 0.107), np.array([[0.707107, -0.707107, 0.0], [0.707107, 0.707107, 0.0],
                                                   [0.0, 0.0, 1.0]])
TCP_POS = (0.0, 0.0, 0.1034)


def rz(q):
    c, s = math.cos(q), math.sin(q)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def kinematics(q):
    """World origins and orientations of links 1..7 and the tcp: (p_tcp, R_tcp, axes z_j, origins p_j)."""
    R, p = np.eye(3), np.zeros(3)  # panda_link0 = world (fixed, base at the origin, setRobot :56-66)
    axes, origins = [], []
    for j in range(DOF):
        p = p + R @ np.array(JOINT_POS[j])
        R = R @ JOINT_ROT[j].T @ rz(q[j])
        axes.append(R[:, 2].copy())
        origins.append(p.copy())
    p = p + R @ np.array(HAND_POS)
    R = R @ HAND_ROT.T
    p = p + R @ np.array(TCP_POS)
    return p, R, axes, origins


def jacobian(q):
    p, R, axes, origins = kinematics(q)
    J = np.zeros((6, DOF))
    for j in range(DOF):
        J[:3, j] = np.cross(axes[j], p - origins[j])
        J[3:, j] = axes[j]
    return J


def manipulability(q):
    J = jacobian(q)
    return math.sqrt(np.linalg.det(J @ J.T))


def d_manipulability(q, delta=1e-4):
    d = np.zeros(DOF)
    for i in range(DOF):
        e = np.zeros(DOF)
        e[i] = delta
        d[i] = (manipulability(q + e) - manipulability(q - e)) / (2 * delta)
    return d


class Mlp:
    """calculateMlpOutput of the reference's NeRF ReLU networks."""

    def __init__(self, par_dir, n_in, n_out, hidden):
        self.n_in = n_in
        dims = [3 * n_in] + list(hidden) + [n_out]
        self.W, self.b = [], []
        for layer in range(len(dims) - 1):
            w = np.loadtxt(os.path.join(par_dir, f"weight_{layer}.txt")).reshape(dims[layer + 1], dims[layer])
            b = np.loadtxt(os.path.join(par_dir, f"bias_{layer}.txt")).reshape(dims[layer + 1])
            self.W.append(w)
            self.b.append(b)

    def __call__(self, x):
        x = np.asarray(x, float)
        nerf = np.concatenate([x, np.sin(x), np.cos(x)])
        jac = np.vstack([np.eye(self.n_in), np.diag(np.cos(x)), -np.diag(np.sin(x))])
        h, d = nerf, jac
        for layer in range(len(self.W) - 1):
            z = self.W[layer] @ h + self.b[layer]
            gate = (z > 0).astype(float)
            d = (gate[:, None] * self.W[layer]) @ d
            h = np.maximum(z, 0.0)
        out = self.W[-1] @ h + self.b[-1]
        return out, self.W[-1] @ d


def load_networks(ref_root):
    nn = os.path.join(ref_root, "cpp", "NNmodel")
    return (Mlp(os.path.join(nn, "self", "parameter"), DOF, 1, [256, 64]),
            Mlp(os.path.join(nn, "env", "parameter"), DOF + 3, NLINK, [256, 256, 256, 256]))


def record(q, obs_xyz, obs_r, nets):
    """RobotData::update + updateEnv for one stage in the REC_* layout of tools/qp_restate.py."""
    import qp_restate as qr
    selfnet, envnet = nets
    q = np.asarray(q, float)
    rec = np.zeros(qr.REC)
    p, R, _, _ = kinematics(q)
    J = jacobian(q)
    rec[qr.REC_POS:qr.REC_POS + 3] = p
    rec[qr.REC_ROT:qr.REC_ROT + 9] = R.reshape(9)
    rec[qr.REC_J:qr.REC_J + 42] = J.reshape(42)
    rec[qr.REC_MU] = math.sqrt(np.linalg.det(J @ J.T))
    rec[qr.REC_DMU:qr.REC_DMU + 7] = d_manipulability(q)
    v, dv = selfnet(q)
    rec[qr.REC_SEL] = v[0]
    rec[qr.REC_DSEL:qr.REC_DSEL + 7] = dv[0]
    rec[qr.REC_OBSR] = obs_r
    v, dv = envnet(np.concatenate([q, np.asarray(obs_xyz, float)]))
    rec[qr.REC_ENV:qr.REC_ENV + 9] = v
    rec[qr.REC_DENV:qr.REC_DENV + 63] = dv[:, :DOF].reshape(63)
    return rec
