// Memory layout of the per-scenario blocks shared by the host wrapper, the C-ABI and the kernels.
// All arrays are fp64, scenario-major (structure of arrays per scenario, scenarios contiguous).
#pragma once

// ---- parameter block (one per scenario), size DAT_PARAM_SIZE(n) doubles -------------------------
// Derived from RQPParameters (reference system/rigid_quadrotor_payload.py:48-84), the equilibrium
// forces f_eq (control/rqp_cadmm.py:165-174) and the controller constants
// (control/rqp_cadmm.py:192-236, control/rqp_centralized.py:182-225).
#define DAT_P_MT 0            // total mass mT
#define DAT_P_XCOM 1          // x_com (3)
#define DAT_P_JT 4            // JT (3x3, row-major)
#define DAT_P_JTI 13          // JT^-1 (3x3)
#define DAT_P_MINFZ 22        // min_fz = mT g / (10 n)
#define DAT_P_MAXF 23         // max_f = 2 mT g / n
#define DAT_P_SEC 24          // sec(max_f_ang)
#define DAT_P_COSP 25         // cos(max_p_ang)
#define DAT_P_MAXWL2 26       // max_wl^2
#define DAT_P_MAXVL2 27       // max_vl^2
#define DAT_P_DISTEPS 28      // dist_eps
#define DAT_P_VISR 29         // vision radius = collision radius + 5
#define DAT_P_COSCONE 30      // cos(vision cone half angle)
#define DAT_P_MAXDEC 31       // max deceleration (g / 5)
#define DAT_P_COLR 32         // capsule (collision) radius
#define DAT_P_KFD 33          // k_f  distributed (0.1 / n)
#define DAT_P_KMD 34          // k_m  distributed
#define DAT_P_KFC 35          // k_f  centralized (0.1)
#define DAT_P_KMC 36          // k_m  centralized
#define DAT_P_KFEQ 37         // k_feq
#define DAT_P_AENVD 38        // alpha_env distributed (1.5)
#define DAT_P_AENVC 39        // alpha_env centralized (2.0)
#define DAT_P_ML 40           // payload mass (informational)
#define DAT_P_HDR 41
#define DAT_P_R(n) (DAT_P_HDR)                    // r (3n): attachment points, body frame, agent-major
#define DAT_P_RCOM(n) (DAT_P_HDR + 3 * (n))      // r_com (3n)
#define DAT_P_FEQ(n) (DAT_P_HDR + 6 * (n))       // f_eq (3n)
#define DAT_P_J(n) (DAT_P_HDR + 9 * (n))         // quad inertias J_i (9n, row-major 3x3 each)
#define DAT_P_JINV(n) (DAT_P_HDR + 18 * (n))     // J_i^-1 (9n)
#define DAT_PARAM_SIZE(n) (DAT_P_HDR + 27 * (n))

// ---- state block (one per scenario), size DAT_STATE_SIZE(n) doubles ------------------------------
// RQPState (reference system/rigid_quadrotor_payload.py:87-119): R_i (9n, row-major 3x3), w_i (3n),
// xl (3), vl (3), Rl (9, row-major), wl (3).  A per-scenario int counter (steps since the last
// polar projection) lives in a separate int array.
#define DAT_S_R(n) 0
#define DAT_S_W(n) (9 * (n))
#define DAT_S_XL(n) (12 * (n))
#define DAT_S_VL(n) (12 * (n) + 3)
#define DAT_S_RL(n) (12 * (n) + 6)
#define DAT_S_WL(n) (12 * (n) + 15)
#define DAT_STATE_SIZE(n) (12 * (n) + 18)

// ---- forest / mountain record (DAT_MOUNTAIN_SIZE doubles) -----------------------------------------
// example/env_forest.py:22-31,74-77: centre (2), radius, sphere radius, centre depth
#define DAT_M_CX 0
#define DAT_M_CY 1
#define DAT_M_RADIUS 2
#define DAT_M_SPHERE_R 3
#define DAT_M_DEPTH 4
#define DAT_MOUNTAIN_SIZE 5

#define DAT_BARK_RADIUS 0.3
#define DAT_BARK_HALF_HEIGHT 2.0
#define DAT_NENV 10            // env CBF rows per QP (control/rqp_cadmm.py:218)
#define DAT_MAXROW 13          // tilt + |wl| + |vl| + 10 env rows
#define DAT_GRAVITY 9.80665    // scipy.constants.g
