/* dat.h -- C-ABI of the MI355X batched agent-QP solver (libdat.so).
 *
 * Drop-in boundary for the reference's controller hot path.  In the reference
 * (AkshayThiru/distributed-aerial-transportation) the plug-in point is the cvxpy solver
 * backend: control/rqp_cadmm.py:16-17 (_RQPCDMM_SOLVER = cv.CLARABEL), control/rqp_dd.py:17-18
 * (_RQPDD_SOLVER) and control/rqp_centralized.py:132,440 (cv.CLARABEL literal), called once per
 * agent QP from RQPPrimalSolver.solve (control/rqp_cadmm.py:482-501, control/rqp_dd.py:475-505)
 * and RQPCentralizedController.control (control/rqp_centralized.py:436-448).  This library
 * replaces that per-call path with batched calls over B independent scenarios; the Python
 * controller classes in distributed_aerial_transportation_amd/control.py keep the reference
 * constructor and control(state, acc_des) signatures on top of it.
 *
 * Conventions: fp64 everywhere; caller-owned, C-contiguous host buffers, read/written only
 * during the call; block layouts in distributed_aerial_transportation_amd/csrc/dat_layout.h;
 * return 0 on success, < 0 on error (message via dat_last_error()); no C++ exceptions cross
 * the ABI.  A handle is bound to one HIP device and one stream and is not re-entrant.
 */
#ifndef DAT_H
#define DAT_H

#ifdef __cplusplus
extern "C" {
#endif

#define DAT_MODE_CENTRALIZED 0 /* RQPCentralizedController  control/rqp_centralized.py:27-455 */
#define DAT_MODE_CADMM 1       /* RQPCADMMController         control/rqp_cadmm.py:510-688    */
#define DAT_MODE_DD 2          /* RQPDDController            control/rqp_dd.py:558-764       */

/* low-level SO(3) attitude law of RQPLowLevelController(so3_controller_type, ...)
 * (control/rqp_centralized.py:457-484) */
#define DAT_LL_PD 0 /* "pd": so3_pd_tracking_control  utils/so3_tracking_controllers.py:18-43 */
#define DAT_LL_SM 1 /* "sm": so3_sm_tracking_control  utils/so3_tracking_controllers.py:52-95 */

/* per agent-QP status (maps the cvxpy/Clarabel outcomes the reference branches on) */
#define DAT_QP_OPTIMAL 0    /* accepted                         (prob.status == OPTIMAL)        */
#define DAT_QP_INACCURATE 1 /* previous solution held           (non-OPTIMAL status)            */
#define DAT_QP_INFEASIBLE 2 /* previous solution held           (non-OPTIMAL status)            */
#define DAT_QP_FAILED 3     /* equilibrium forces used          (solver exception, :491-494)    */

typedef struct dat_handle dat_handle;

typedef struct dat_config {
  int device;        /* HIP device ordinal                                               */
  int mode;          /* DAT_MODE_*                                                       */
  int n;             /* quadrotors per payload (3 <= n <= 16)                            */
  int batch;         /* number of independent scenarios B                                */
  double dt;         /* simulation step [s] (example/rqp_example.py:85: 1e-3)            */
  int hl_every;      /* simulation steps per high-level step (rqp_example.py:86: 10)     */
  int max_iter;      /* ADMM/DD max_iter (control/rqp_cadmm.py:563: 100)                 */
  double res_tol;    /* ADMM/DD residual tolerance (control/rqp_cadmm.py:561: 1e-2)      */
  int use_total_res; /* C-ADMM residual kind (control/rqp_cadmm.py:562: 1)               */
  double rho0, tau_incr, rho_max; /* C-ADMM penalty schedule (control/rqp_cadmm.py:565-567) */
  int record_err;    /* keep per-iteration residual sequences (SolverStatistics.err_seq) */
} dat_config;

/* ---- lifecycle ------------------------------------------------------------------------- */
/* dat_create replaces the controller constructors (RQPCADMMController.__init__
 * control/rqp_cadmm.py:513-538, RQPDDController.__init__ control/rqp_dd.py:561-586,
 * RQPCentralizedController.__init__ control/rqp_centralized.py:46-132): it allocates the
 * persistent warm state the reference keeps in Python objects (f, f_mean, lambda
 * control/rqp_cadmm.py:569-580; lambda_F, lambda_M control/rqp_dd.py:618-632; prev_f). */
void dat_default_config(dat_config* cfg);
int dat_create(const dat_config* cfg, dat_handle** out);
int dat_destroy(dat_handle* h);
const char* dat_last_error(void); /* thread-local message of the last failing call */
int dat_device_count(void);

/* ---- problem data ------------------------------------------------------------------------ */
/* params: per_scenario ? B x DAT_PARAM_SIZE(n) : DAT_PARAM_SIZE(n) (broadcast).  The block holds
 * RQPParameters' derived fields (system/rigid_quadrotor_payload.py:48-84), f_eq
 * (_set_system_constants, control/rqp_cadmm.py:142-190) and the controller constants
 * (_set_controller_constants, control/rqp_cadmm.py:192-236, rqp_centralized.py:182-225).
 * Resets the warm state to the constructor's (f = f_eq, lambda = 0). */
int dat_set_params(dat_handle* h, const double* params, int per_scenario);
/* forests: num_forests layouts; tree_offsets[num_forests+1] index rows of tree_pos (T x 3; the handle keeps each forest sorted by x);
 * scenario_forest[B] selects a layout per scenario (NULL: all use layout 0, -1: no env);
 * mountain[num_forests x DAT_MOUNTAIN_SIZE] for the desired-acceleration law.  num_forests = 0
 * removes the environment (env = None in the reference). */
/* Replaces the env object handed to the controllers (Forest, example/env_forest.py:35-85) and the
 * hppfcl queries made through it (centralized_distance / distributed_distance :139-212). */
int dat_set_forests(dat_handle* h, int num_forests, const int* tree_offsets, const double* tree_pos,
                    const int* scenario_forest, const double* mountain);
/* set_force_err_tolerance: control/rqp_cadmm.py:683-685, control/rqp_dd.py:760-761 */
int dat_set_tolerance(dat_handle* h, double res_tol, int use_total_res);
/* Stopping tolerance of every agent / centralized QP's interior-point solve (default 1e-10).  The
 * reference solves with Clarabel's default settings (prob.solve(solver=CLARABEL), control/rqp_cadmm.py:492,
 * control/rqp_dd.py:485, control/rqp_centralized.py:440: tol_gap_abs = tol_gap_rel = tol_feas = 1e-8);
 * 1e-8 here is that tolerance.  tol in [1e-12, 1e-7] (the north_star residual bound), else an error. */
int dat_set_qp_tolerance(dat_handle* h, double tol);
/* set_max_iter: control/rqp_cadmm.py:687-688, control/rqp_dd.py:763-764 */
int dat_set_max_iter(dat_handle* h, int max_iter);
/* _set_warm_start: control/rqp_cadmm.py:577-580, control/rqp_dd.py:628-632 */
int dat_reset_warm_start(dat_handle* h);

/* ---- state ------------------------------------------------------------------------------ */
int dat_set_state(dat_handle* h, const double* state /* B x DAT_STATE_SIZE(n) */, const int* counters /* B or NULL */);
int dat_get_state(dat_handle* h, double* state, int* counters);

/* ---- one high-level control step for every scenario ---------------------------------------
 * Replaces controller.control(state, acc_des) -> (f_des, SolverStatistics):
 *   RQPCADMMController.control   control/rqp_cadmm.py:631-675  (agent solves :482-501)
 *   RQPDDController.control      control/rqp_dd.py:695-752     (agent solves :475-505)
 *   RQPCentralizedController.control control/rqp_centralized.py:436-448
 * state: B x DAT_STATE_SIZE(n) or NULL (use the device-resident state);
 * acc_des: B x 6 (dvl_des, dwl_des) or NULL (forest law example/rqp_example.py:33-59 on device).
 * Outputs (any may be NULL): f_des B x 3n (agent-major, the forces the controller returns),
 * iters B (SolverStatistics.iter; -1 for centralized), qp_status B x n (last solve per agent),
 * min_env_dist B, collision B, err_seq B x (max_iter+1) (NaN padded; needs record_err). */
int dat_control_step(dat_handle* h, const double* state, const double* acc_des, double* f_des, int* iters,
                     int* qp_status, double* min_env_dist, unsigned char* collision, double* err_seq);

/* ---- fused control steps (QP-level workloads: C-ADMM / DD handles without a forest): `steps`
 * consecutive control steps of every scenario from the resident states, scenario s's step k using
 * acc_seq[(k B + s) x 6 ..] -- the same arithmetic per scenario as `steps` calls of dat_control_step
 * (warm f, f_mean, lambda / lambda_F, lambda_M carried; control/rqp_cadmm.py:631-675,
 * control/rqp_dd.py:695-752), in ONE persistent drain: a scenario that finishes step k starts step
 * k + 1 in its slot at once instead of waiting for the slowest scenario of step k.  Outputs (optional,
 * NULL to skip) are those of the last step.  record_err must be 0. */
int dat_control_steps(dat_handle* h, int steps, const double* acc_seq, double* f_des, int* iters, int* qp_status);

/* ---- rollout: `steps` simulation steps (SO(3) PD low level + rigid-body dynamics) ---------
 * Replaces RQPLowLevelController.control (control/rqp_centralized.py:518-535) followed by
 * RQPDynamics.integrate (system/rigid_quadrotor_payload.py:271-276) per simulation step.
 * f_des: B x 3n held constant over the steps, or NULL to use the last control step's output. */
int dat_rollout(dat_handle* h, int steps, const double* f_des);
/* Low-level law used by dat_rollout / dat_closed_loop: DAT_LL_PD (default, example/rqp_example.py:113)
 * or DAT_LL_SM -- the so3_controller_type argument of RQPLowLevelController (control/rqp_centralized.py:468-482). */
int dat_set_low_level(dat_handle* h, int kind);
/* RQPLowLevelController.control(state, f_des) -> (f, M) (control/rqp_centralized.py:518-535) at the
 * current states: f_des B x 3n (agent-major) or NULL (the last control step's output); thrust B x n,
 * moment B x n x 3 (agent-major 3-vectors). */
int dat_low_level_control(dat_handle* h, const double* f_des, double* thrust, double* moment);
/* Rigid payload driven by actuator forces (RPDynamics.integrate, system/rigid_payload.py:93-172): `steps`
 * steps of dt on the payload part of the states (xl, vl, Rl, wl; Rl projected every 20 steps), forces
 * f B x 3n (agent-major, ground frame; NULL: the last control step's output) held.  The handle carries
 * the rigid-payload parameter block (rigid_payload.pack_rp_params: mT = ml, JT = Jl, r_com = r), whose
 * centralized QP is RPCentralizedController (control/rp_centralized.py:9-306) via dat_control_step. */
int dat_rp_rollout(dat_handle* h, int steps, const double* f);

/* ---- device-resident closed loop (the loop of example/rqp_example.py:120-131 with the desired
 * acceleration of :33-59): hl_steps x (desired acceleration + control step +
 * hl_every rollout steps); inputs already in HBM, nothing copied per step. */
int dat_closed_loop(dat_handle* h, int hl_steps);
/* C-ADMM handles: run dat_closed_loop on `count` (1..4) contiguous sub-batches of the scenarios, each on
 * its own stream with no synchronisation between sub-batches or steps, so that one sub-batch's kernels
 * fill the others' drain tails and short kernels.  Per scenario the arithmetic is unchanged (a scenario's
 * results never depend on the grouping).  count = 1 (default) restores the single-stream loop.  With a forest
 * and count = 1 the scenarios wedged in a stall (previous step > TAIL_PREV ADMM passes) run in the tail kernel
 * on a second stream beside the drain; with count > 1 (no further stream: the device's hardware queues are
 * shared by all streams) the drain hands them to the tail kernel before their first pass -- the same passes,
 * the same results. */
int dat_set_sub_batches(dat_handle* h, int count);
/* Host steady-clock marks (ms) of the last dat_closed_loop call: [0] its start (0.0), then the completion
 * of each HL step's control kernel; consecutive differences are per-step times of the back-to-back run.
 * Writes up to max_marks values; returns the number of marks (hl_steps + 1).  With sub-batch streams
 * (dat_set_sub_batches > 1) the steps of different sub-batches overlap: only the start and the end of the
 * run are marked (2 marks), so consecutive differences give one whole-run time, not per-step times. */
int dat_get_step_marks(dat_handle* h, double* marks_ms, int max_marks);

/* ---- counters since the last reset: agent-QP solves, IPM iterations, IPM iterations x active
 * constraint rows (for the flop model of DESIGN.md 3.1), control steps, and the summed device time
 * of the high-level kernels [ms] (HIP events on the handle stream).  Any pointer may be NULL. */
int dat_get_counters(dat_handle* h, long long* qp_solves, long long* ipm_iters, long long* ipm_row_iters,
                     long long* hl_steps, double* hl_kernel_ms);
/* C-ADMM only: the same counters for one env class and the summed device time of k_cadmm [ms]
 * (one persistent launch drains every class).  env_class in [0, 4): scenarios whose agent QPs carry
 * no env CBF row this step (0), or at most 2 (1), 5 (2), 10 (3) env rows per agent QP. */
int dat_get_class_counters(dat_handle* h, int env_class, long long* qp_solves, long long* ipm_iters,
                           long long* ipm_row_iters, double* kernel_ms);
/* C-ADMM only, SIMD occupancy of one env class: slot_ipm_iters = sum over wavefront ADMM passes of
 * (the largest IPM iteration count among the wavefront's lanes) x lanes in use, wave_admm_iters =
 * sum over wavefronts of ADMM passes x scenarios per wavefront.  ipm_iters / slot_ipm_iters is the
 * fraction of lane-iterations doing useful work (the rest idle on divergence). */
int dat_get_class_occupancy(dat_handle* h, int env_class, long long* slot_ipm_iters, long long* wave_admm_iters);
int dat_reset_counters(dat_handle* h);
int dat_synchronize(dat_handle* h);
/* C-ADMM / DD: number of resident k_cadmm / k_dd workgroups that drain the scenario queues (0 = default,
 * 4 x CUs).  A scenario's arithmetic does not depend on it; tests cap it at 1-2 workgroups so that
 * scenario slots are refilled many times within one control step. */
int dat_set_persistent_blocks(dat_handle* h, int blocks);
/* Summed device time [ms] since the last counter reset of the main solver kernel of each control step:
 * k_cadmm (C-ADMM) or k_dd (DD; the per-scenario quasi-Newton setup k_dd_setup excluded), 0 for
 * centralized.  Both are persistent queue drains; dat_set_persistent_blocks caps their grid.  A closed
 * loop on S sub-batches (dat_set_sub_batches) launches k_cadmm S times per HL step, one per sub-batch:
 * the sum then covers hl_steps x S launches. */
int dat_get_kernel_ms(dat_handle* h, double* ms);
/* Agent QPs since the last counter reset (every kernel) that stalled before the IPM tolerance (1e-10:
 * a numerical breakdown of the structured Newton solve at gaps ~1e-12, or the divergence stop) and
 * were accepted as OPTIMAL through their best iterate inside north_star's band (scaled primal / dual
 * residuals <= 1e-7, gap <= 1e-6); beyond_clarabel_tol counts those whose returned iterate is outside
 * Clarabel's own stopping tolerance (1e-8: a point Clarabel would not yet report as solved).  The
 * reference holds its previous solution on a non-OPTIMAL status (control/rqp_cadmm.py:496-499), so
 * beyond_clarabel_tol bounds the branch-disagreement risk; the C-ADMM / DD parity tests require 0. */
int dat_get_inband_exits(dat_handle* h, long long* inband, long long* beyond_clarabel_tol);
/* IPM iterative-refinement passes run and corrections applied by every kernel since the last counter
 * reset: the executed-work terms of the flop model. */
int dat_get_refinement_counters(dat_handle* h, long long* passes, long long* corrections);
/* C-ADMM control steps of a scenario finished by the tail kernel since the last counter reset: k_cadmm
 * hands a scenario's step to k_cadmm_tail, at the ADMM pass it is in, when one of its agent QPs does not
 * end cleanly (INACCURATE, or accepted in band beyond Clarabel's 1e-8: inside the reference's max_iter
 * stalls next to trees) or, with a forest, when the tail rule holds for its next pass (the previous step took
 * more than 20 ADMM passes, or the pass is the 16th); k_env_class routes a scenario whose previous step took
 * more than 20 passes to the tail before the step.  k_cadmm_tail redoes unclean QPs with the robust solver
 * (stiff rows in augmented form) and finishes the step.  Replaces no reference call (Clarabel's internal KKT
 * regularisation); the per-QP surfaces (dat_solve_agent_qp_batch) redo the QP themselves. */
int dat_get_robust_redos(dat_handle* h, long long* redos);
/* The tail kernel's work since the last counter reset (out[6]): [0] ADMM passes, [1] the sum over its passes of
 * the slowest agent QP's IPM iterations (the critical path of the stalled steps), [2] scenario-steps routed to
 * the tail before the step, [3] agent QPs whose rows were certified infeasible (a Farkas certificate on the dvl
 * rows: the QP is held at its previous solution, as the reference holds it when Clarabel reports infeasible,
 * control/rqp_cadmm.py:496-499), [4] solves ended by the stall exit, [5] warm-started solves.  Replaces no
 * reference call. */
int dat_get_tail_counters(dat_handle* h, long long* out);
/* C-ADMM with a forest: scenario-steps with a collision flag and the smallest minimum env distance over every
 * HL step since the last counter reset, signed (negative once a body is inside a tree: the reference logs
 * min_env_dist per step and flags a collision below its threshold: example/rqp_example.py:129,
 * example/env_forest.py:158-159; +inf without a forest). */
int dat_get_collision_stats(dat_handle* h, long long* collisions, double* min_env_dist);
/* Device time [ms] of the last dat_solve_agent_qp_batch launch (k_agent_qp; HIP events on the handle's
 * stream): the solve_time RQPPrimalSolver.solve returns (Clarabel's solver_stats.solve_time,
 * control/rqp_cadmm.py:500, control/rqp_dd.py:497). */
int dat_get_agent_qp_ms(dat_handle* h, double* ms);

/* ---- raw batched kernels (tests / benchmarking of single pieces) ---------------------------
 * dat_env_rows: _set_collision_avoidance_cbf_parameters (control/rqp_cadmm.py:307-373,
 * control/rqp_centralized.py:280-337) for every (scenario, agent).
 * Env CBF rows for every (scenario, agent) of the current state: lhs B x n x 10 x 3, rhs
 * B x n x 10, nrow B x n, collision B x n, min_dist B x n (agent = -1 row when centralized). */
int dat_env_rows(dat_handle* h, double* lhs, double* rhs, int* nrow, unsigned char* collision, double* min_dist);

/* dat_solve_agent_qp_batch: `count` independent agent QPs -- RQPPrimalSolver.solve
 *   C-ADMM handles: solve(state, acc_des, lambda_f, cadmm_rho, f_mean) -> f   control/rqp_cadmm.py:482-501
 *   DD handles:     solve(state, acc_des, c_fi, c_Fi, c_Mi) -> (f_i, F_i, M_i) control/rqp_dd.py:475-505
 * at the handle's current states (dat_set_state), parameters and forests.  Item k: scenario[k],
 * agent[k], acc_des[6k..] (dvl_des, dwl_des) and
 *   C-ADMM: lam[3n k ..] (lambda_f, agent-major 3-vectors), rho[k] > 0, f_mean[3n k ..];
 *   DD:     c9[9k ..] = (c_fi, c_Fi, c_Mi)  (lam, rho, f_mean unused; NULL allowed).
 * Outputs: x[3n k ..] (C-ADMM: agent i's full copy f, agent-major) or x[9k ..] (DD: f_i, F_i, M_i),
 * status[k] (DAT_QP_*), and, if not NULL, ipm_iters[k], collision[k], min_env_dist[k] of the agent's
 * env query (control/rqp_cadmm.py:307-373).  A non-OPTIMAL item returns the IPM's best iterate; the
 * reference's fallbacks (hold previous / f_eq, :491-499) are the caller's (RQP*PrimalSolver in
 * control.py).  No warm state is read or written. */
int dat_solve_agent_qp_batch(dat_handle* h, int count, const int* scenario, const int* agent, const double* acc_des,
                             const double* lam, const double* rho, const double* f_mean, const double* c9, double* x,
                             int* status, int* ipm_iters, unsigned char* collision, double* min_env_dist);

/* ---- metric collectives of a sharded run (K8) ----------------------------------------------
 * Scenarios shard over the GPUs of a node with no collective inside the control step; what crosses GPUs is the
 * per-scenario metrics the reference's loop keeps in its lists (iteration counts, min env distance, collision
 * flag: example/rqp_example.py:112-138) and the run's work counters.  The reference runs one scenario in one
 * process and has no such call; these replace the torch.distributed collectives a PyTorch harness would use,
 * over RCCL (xGMI), with host buffers.  One process per GPU: rank 0 creates the id, the launcher hands it to the
 * others (sharding.py: a file keyed by the launcher's rendezvous), every rank calls dat_comm_create. */
#define DAT_COMM_ID_BYTES 128
#define DAT_COMM_SUM 0
#define DAT_COMM_MAX 1
typedef struct dat_comm dat_comm;
int dat_comm_unique_id(unsigned char* id /* DAT_COMM_ID_BYTES */);
int dat_comm_create(int device, int nranks, int rank, const unsigned char* id, dat_comm** out);
int dat_comm_destroy(dat_comm* c);
/* recv[nranks x count] = every rank's send[count], in rank order */
int dat_comm_allgather(dat_comm* c, const double* send, long long count, double* recv);
/* buf[count] = element-wise sum (DAT_COMM_SUM) or max (DAT_COMM_MAX) over the ranks, in place */
int dat_comm_allreduce(dat_comm* c, double* buf, long long count, int op);
/* every rank's device work done, then a one-value all-reduce */
int dat_comm_barrier(dat_comm* c);
const char* dat_comm_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* DAT_H */
