// host_params.cpp — Params/*.json loaders with the reference's ParamValue override semantics.
//
// Restates Param / CostParam / BoundsParam / NormalizationParam / SQPParam (params.cpp:24-448) and
// resolves which consumer sees which value, as the reference's constructors do:
//   MPC(Ts, path, pv)          mpc.cpp:40-52      Param(path, pv.param) for MPC and the track spline
//   OsqpInterface(Ts, path, pv) osqp_interface.cpp:50-59
//       Cost(path, pv)          -> model + cost overrides
//       Constraints(path, pv)   -> model overrides
//       Bounds(BoundsParam(path.bounds_path), Param(path, pv.param))  -> bounds file only (!)
//       NormalizationParam(path, pv.normalization), SQPParam(path, pv.sqp)
//       cost_param_(path.cost_path) -> r_ddq of the QP never overridden (Q8)
//   MPC::setParam / OsqpInterface::setParam (mpc.cpp:204-209, osqp_interface.cpp:95-100): refresh
//       Cost, Constraints, Bounds, MPC::param_; normalization and SQP keep their values, and the
//       track spline's projection distance keeps its construction value.
#include <cstring>
#include <vector>
#include <stdexcept>
#include <string>

#include "host_json.h"
#include "mpcc_engine.h"

namespace mpcc {
void set_last_error(const std::string& m);
}

using namespace mpcc;

namespace {

struct Sections {
    JVal model, cost, bounds, norm, sqp, config;
    bool has_config = false;
};

Sections load_sections(const mpcc_json_paths* p) {
    Sections s;
    if (p->merged_path) {
        JVal m = json_load_file(p->merged_path);
        s.model = m.at("model"); s.cost = m.at("cost"); s.bounds = m.at("bounds");
        s.norm = m.at("normalization"); s.sqp = m.at("sqp");
        if (m.has("config")) { s.config = m.at("config"); s.has_config = true; }
        if (m.has("robot") && m.at("robot").has("mount")) {  // the mount is compiled in (MPCC_MOBILE_MOUNT_Z)
            const std::vector<double> mt = m.at("robot").at("mount").numbers();
            const double want[3] = {0.0, 0.0, MPCC_DOF == 10 ? MPCC_MOBILE_MOUNT_Z : 0.0};
            if (mt.size() != 3 || mt[0] != want[0] || mt[1] != want[1] || mt[2] != want[2])
                throw std::runtime_error("robot.mount differs from the library's compiled mount (0, 0, " +
                                         std::to_string(want[2]) + "); it is part of the robot definition "
                                         "(MPCC_MOBILE_MOUNT_Z, include/mpcc_engine.h): rebuild to change it");
        }
    }
    if (p->param_path) s.model = json_load_file(p->param_path);
    if (p->cost_path) s.cost = json_load_file(p->cost_path);
    if (p->bounds_path) s.bounds = json_load_file(p->bounds_path);
    if (p->normalization_path) s.norm = json_load_file(p->normalization_path);
    if (p->sqp_path) s.sqp = json_load_file(p->sqp_path);
    return s;
}

struct Overrides {
    const mpcc_override* ov;
    int n;
    // value of key in section, or the file value
    double get(const JVal& file, const char* section, const char* key) const {
        for (int i = 0; i < n; i++)
            if (ov[i].section && ov[i].key && std::strcmp(ov[i].section, section) == 0 && std::strcmp(ov[i].key, key) == 0)
                return ov[i].value;
        return file.at(key).number();
    }
};

}  // namespace

extern "C" int mpcc_params_load_json(const mpcc_json_paths* paths, const mpcc_override* overrides, int n_overrides,
                                     int ctor_semantics, int N, mpcc_params* out) {
    if (!paths || !out || N < 1) {
        set_last_error("mpcc_params_load_json: invalid argument");
        return MPCC_E_INVALID;
    }
    try {
        Sections s = load_sections(paths);
        Overrides o{overrides, overrides ? n_overrides : 0};
        Overrides none{nullptr, 0};
        mpcc_params p;
        std::memset(&p, 0, sizeof p);
        p.N = N;
        p.Ts = s.has_config && s.config.has("Ts") ? s.config.at("Ts").number() : 0.01;
        p.constraint_mask = MPCC_CON_SELFCOL | MPCC_CON_SING | MPCC_CON_ENVCOL;
        // Param (model.json), overridable
        const JVal& m = s.model;
        p.proj_max_dist = o.get(m, "param", "max_dist_proj");
        p.guess_max_dist = p.proj_max_dist;
        p.desired_ee_velocity = o.get(m, "param", "desired_ee_velocity");
        p.deacc_ratio = o.get(m, "param", "deaccelerate_ratio");
        p.cost_tol_selcol = o.get(m, "param", "tol_selcol");
        p.cost_tol_sing = o.get(m, "param", "tol_sing");
        p.con_tol_selcol = p.cost_tol_selcol;
        p.con_tol_sing = p.cost_tol_sing;
        p.con_tol_envcol = o.get(m, "param", "tol_envcol");
        p.s_trust_region = o.get(m, "param", "s_trust_region");
        // CostParam (cost.json), overridable for Cost
        const JVal& c = s.cost;
        p.q_c = o.get(c, "cost", "qC");
        p.q_c_N_mult = o.get(c, "cost", "qCNmult");
        p.q_l = o.get(c, "cost", "qL");
        p.q_vs = o.get(c, "cost", "qVs");
        p.q_ori = o.get(c, "cost", "qOri");
        p.q_sing = o.get(c, "cost", "qSing");
        p.r_dq = o.get(c, "cost", "rdq");
        p.r_dVs = o.get(c, "cost", "rdVs");
        p.q_c_red_ratio = o.get(c, "cost", "qC_reduction_ratio");
        p.q_l_inc_ratio = o.get(c, "cost", "qL_increase_ratio");
        p.q_ori_red_ratio = o.get(c, "cost", "qOri_reduction_ratio");
        p.qp_r_ddq = none.get(c, "cost", "rddq");  // Q8
        // BoundsParam: always the file (osqp_interface.cpp:54, 99)
        const JVal& b = s.bounds;
        // joint names: the Husky base joints (xb, yb, thb; mobile_params.json) precede the Panda joints
        const char* qn_all[10] = {"xb", "yb", "thb", "q1", "q2", "q3", "q4", "q5", "q6", "q7"};
        const char* dn_all[10] = {"dxb", "dyb", "dthb", "dq1", "dq2", "dq3", "dq4", "dq5", "dq6", "dq7"};
        const char* const* qn = qn_all + (10 - MPCC_DOF);
        const char* const* dn = dn_all + (10 - MPCC_DOF);
        const int XS = MPCC_DOF, XVS = MPCC_DOF + 1, UVS = MPCC_DOF;
        for (int j = 0; j < MPCC_DOF; j++) {
            p.lx[j] = b.at(std::string(qn[j]) + "l").number();
            p.ux[j] = b.at(std::string(qn[j]) + "u").number();
            p.lu[j] = b.at(std::string(dn[j]) + "l").number();
            p.uu[j] = b.at(std::string(dn[j]) + "u").number();
            p.lddq[j] = b.at(std::string("d") + dn[j] + "l").number();
            p.uddq[j] = b.at(std::string("d") + dn[j] + "u").number();
        }
        p.lx[XS] = b.at("sl").number(); p.ux[XS] = b.at("su").number();
        p.lx[XVS] = b.at("vsl").number(); p.ux[XVS] = b.at("vsu").number();
        p.lu[UVS] = b.at("dVsl").number(); p.uu[UVS] = b.at("dVsu").number();
        // NormalizationParam, SQPParam: overrides only with constructor semantics
        const Overrides& on = ctor_semantics ? o : none;
        const JVal& nn = s.norm;
        for (int j = 0; j < MPCC_DOF; j++) p.Tx[j] = on.get(nn, "normalization", qn[j]);
        p.Tx[XS] = on.get(nn, "normalization", "s");
        p.Tx[XVS] = on.get(nn, "normalization", "vs");
        for (int j = 0; j < MPCC_DOF; j++) p.Tu[j] = on.get(nn, "normalization", dn[j]);
        p.Tu[UVS] = on.get(nn, "normalization", "dVs");
        const JVal& q = s.sqp;
        p.eps_prim = on.get(q, "sqp", "eps_prim");
        p.eps_dual = on.get(q, "sqp", "eps_dual");
        p.line_search_tau = on.get(q, "sqp", "line_search_tau");
        p.line_search_eta = on.get(q, "sqp", "line_search_eta");
        p.line_search_rho = on.get(q, "sqp", "line_search_rho");
        p.max_iter = (int32_t)on.get(q, "sqp", "max_iter");
        p.line_search_max_iter = (int32_t)on.get(q, "sqp", "line_search_max_iter");
        p.do_SOC = on.get(q, "sqp", "do_SOC") != 0.0;
        p.use_BFGS = on.get(q, "sqp", "use_BFGS") != 0.0;
        p.vio_floor = 1e-9;
        *out = p;
        return MPCC_OK;
    } catch (const std::exception& e) {
        set_last_error(std::string("mpcc_params_load_json: ") + e.what());
        return MPCC_E_IO;
    }
}
