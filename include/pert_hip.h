/* pert_hip.h -- C ABI of the MI355X PERT hot path (libpert_hip.so, gfx950).
 *
 * The reference has no FFI: its replaceable unit is Pyro's
 *   svi.step(gammas, libs, data=..., etas=..., lamb=..., t_init=...) -> float
 * (scdna_replication_tools/pert_model.py:743 step 1, :801 step 2, :868 step 3)
 * plus the MAP decode infer_discrete(temperature=0) (:762-769, :820-827, :886-893).
 * One SVI step of this library is the launch sequence
 *   pert_enum_pass(PERT_MODE_STEP)   (steps 2/3)  or  pert_obs_pass()  (step 1)
 *   pert_finalize()                  per-cell / per-bin / global gradient reductions
 *   [all-reduce of the shared gradient block across ranks, from the host]
 *   pert_adam()                      Adam on the packed non-pi parameters
 * and the decode is pert_enum_pass(PERT_MODE_DECODE).  With the three-wave pass (variant 3)
 * a step of steps 2/3 is instead pert_enum_step() [+ all-reduce + pert_adam_shared()].
 *
 * Conventions: every buffer is device memory owned by the caller (allocated via
 * the torch caching allocator on the caller's side); nothing here allocates.  All
 * launches go on the caller's stream.  Entry points return 0 on success, a
 * positive PERT_E* code for an argument error and 1000 + hipError_t for a launch
 * failure.  A NaN loss is returned as data (pert_model.py:755-758), never raised.
 *
 * Layouts (bin-major like the reference's (loci x cells) tensors, pert_model.py:156-166);
 * ldn = N rounded up to a multiple of 256 (PERT_BLOCK); padded cells are never stored:
 *   reads      float  [L][ldn]     integer-valued counts
 *   gcf        float  [L][K1]      [gc^K .. gc^1, 1] (make_gc_features, pert_model.py:460-463)
 *   eta_code   uint16 [L][ldn]     row index into eta_table          (steps 2/3)
 *   eta_table  float  [n_codes][P+2]  eta_k - 1 for k < P, then S1 = sum_k (eta_k - 1), then
 *                                   A = fp32 lgamma(sum_k eta_k) as torch evaluates it: each
 *                                   element's Dirichlet value is rounded to A's grid as the
 *                                   reference's fp32 log_prob rounds it (0: not rounded)
 *   z_pi/m_pi/v_pi/g_pi float [ldn/64][L][P][64]  softmax logits of expose_pi and Adam
 *                                   moments in wave tiles: cell n, state k of bin l at
 *                                   (((n/64)*L + l)*P + k)*64 + n%64  (a wave streams one
 *                                   contiguous run over its bins)
 *   cn_obs/rep_obs, cn_out/rep_out uint8 [L][ldn]
 *   packed params (unconstrained, see pert_layout below), float
 *
 * Step 1 pair mode (rep_obs == NULL): the training set of pert_model.py:228-251 -- every
 * G1/2 cell twice, rep 0 then rep 1, same reads and CN -- stored once: N is even, cells
 * [0, N/2) are the rep-0 copies and [N/2, N) the rep-1 copies of the N/2 columns that reads
 * and cn_obs hold, whose row stride ldn (>= N/2, multiple of 256) is that of the stored
 * arrays.  Parameters, libs, mean_reads, ploidy and the workspace stay per cell (N).
 */
#ifndef PERT_HIP_H
#define PERT_HIP_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PERT_KIND_STEP1 1   /* G1/2 cells, cn/rep observed (pert_model.py:718-774) */
#define PERT_KIND_STEP2 2   /* S cells, cn x rep enumerated (:776-830) */
#define PERT_KIND_STEP3 3   /* step 2 with rho, a frozen, on G1 cells (:834-896) */

#define PERT_MODE_STEP   0  /* ELBO + grads + fused Adam on pi + reduction partials */
#define PERT_MODE_GRAD   1  /* ELBO + grads; d(-ELBO)/dz_pi written to g_pi, no update */
#define PERT_MODE_DECODE 2  /* joint argmax over (rep, cn): cn_out, rep_out */

#define PERT_OK 0
#define PERT_E_ARG 1
#define PERT_E_UNSUPPORTED_P 2
#define PERT_E_UNSUPPORTED_K 3
#define PERT_E_COMM_UNAVAILABLE 5   /* RCCL not loaded (pert_comm_load) or lacks a symbol */
#define PERT_E_COMM_ABORTED 6       /* a rank of the fit failed and raised the abort word */
#define PERT_E_COMM_TIMEOUT 7       /* a peer did not arrive within the communicator's deadline */
#define PERT_E_COMM_FAULT 8         /* injected by pert_comm_inject_fault (tests) */
#define PERT_E_HIP_BASE 1000        /* + hipError_t */
#define PERT_E_COMM_BASE 2000       /* + ncclResult_t */

#define PERT_MAX_K1 8      /* K + 1 <= 8 */
#define PERT_MIN_P 2
#define PERT_MAX_P 16
#define PERT_BLOCK 256     /* cells per workgroup (4 waves x 64 lanes) */

/* Offsets into the packed parameter / gradient vectors.  The shared block
 * [0, n_shared) is replicated on every rank and its gradient is all-reduced;
 * the cell block [n_shared, n_params) is local to the rank's cell shard. */
typedef struct {
  int32_t off_rho;     /* L    z_rho (unit interval)                          */
  int32_t off_a;       /* 1    z_a   (positive)                               */
  int32_t off_lam;     /* 1    z_lambda (interval(0.001, 0.999)), step 1      */
  int32_t off_bstds;   /* n_libs*K1  z_beta_stds (positive)                   */
  int32_t off_bmeans;  /* n_libs*K1  beta_means (real), step 1                */
  int32_t n_shared;
  int32_t off_u;       /* N    u (real)                                        */
  int32_t off_beta;    /* K1*N betas, plane layout [k][n]                      */
  int32_t off_tau;     /* N    z_tau (unit interval)                           */
  int32_t n_params;
} pert_layout;

typedef struct {
  int32_t kind, L, N, P, K1, n_libs, n_codes;
  int32_t ldn;                     /* row stride (cells) of every [L][*] array: N rounded up to 256 */
  int32_t is_root;                 /* adds the global priors once across ranks */
  const float* reads;
  const float* gcf;
  const int32_t* libs;             /* [N] library index per cell */
  const uint16_t* eta_code;        /* steps 2/3 */
  const float* eta_table;
  const uint8_t* cn_obs;           /* step 1 */
  const uint8_t* rep_obs;
  const float* mean_reads;         /* [N] mean over bins of reads (u prior, :597) */
  const float* ploidy;             /* [N] mean argmax eta (steps 2/3) or 2 (step 1) */
  float lamb;                      /* steps 2/3: fixed lambda from step 1 */
  float log1m_lam;                 /* log(1 - lamb) */
  double sum_reads;                /* step 1: sum of reads of this shard (d/dlam of x log lam), fp64 */
  float a_fixed;                   /* step 3 */
  const float* beta_means;         /* steps 2/3 fixed [n_libs][K1] */
  const float* rho_fixed;          /* step 3 [L] constrained */
} pert_problem;

typedef struct {
  pert_layout lay;
  float* params;                   /* [n_params] unconstrained */
  float* adam_m;                   /* [n_params] */
  float* adam_v;                   /* [n_params] */
  double* grad_shared;             /* [n_shared + 1]: d loss / d shared params, then loss (local sum) */
  float* grad_cell;                /* [n_params - n_shared] */
  float* z_pi;                     /* [ldn/64][L][P][64] steps 2/3 */
  float* m_pi;
  float* v_pi;
  float* g_pi;                     /* [ldn/64][L][P][64] only for PERT_MODE_GRAD */
  uint8_t* cn_out;                 /* [L][ldn] PERT_MODE_DECODE */
  uint8_t* rep_out;
  /* workspace, sized by pert_workspace_sizes() */
  float* cell_part;
  float* bin_part;
  double* blk_part;
  double* cellblk_part;
  int32_t bins_per_tile;           /* LT; 0 = library default */
  int32_t variant;                 /* enumerated-pass kernel: 0 LDS-DMA streamed (two waves per SIMD),
                                      2 = variant 0 + wave timeline stamps into g_pi (diagnostic, STEP mode),
                                      3 = three waves per SIMD, online logsumexp (pert_enum_step);
                                      anything else (1 was retired in round 3) -> PERT_E_ARG */
  /* Device-side SVI loop control (the loop of pert_model.py:742-758, :800-816, :867-883).
   * loop_ctl == NULL disables it.  Otherwise pert_adam records the loss of iteration
   * `step` (after the cross-rank all-reduce) into loop_rec and evaluates the reference's
   * stopping rule on the device: rel-tol plateau once step >= min_iter (:749-753), then
   * NaN (:755-758); on a stop it sets loop_ctl[0] = step.  Every PERT_MODE_STEP /
   * obs / finalize / adam launch of a later step is then a no-op, so the host can queue
   * iterations ahead without a per-step synchronisation and the fit still stops after
   * exactly the iteration the reference stops after. */
  int32_t* loop_ctl;               /* [2]: stop_at (-1 while running), reason (1 rel_tol, 2 NaN) */
  double* loop_rec;                /* [max_iter][2]: loss of each step, stop_at after it */
  const double* loss_offset;       /* [max_iter] or NULL: per-step loss term kept on the host side
                                      of the ABI (step 1's canonical pi block) */
  double loss_const;               /* loss = grad_shared[n_shared] - loss_const - loss_offset[step] */
  double rel_tol;
  int32_t min_iter;
  int32_t step;                    /* 0-based iteration index of this launch sequence */
} pert_state;

typedef struct {
  float lr, beta1, beta2, eps;
  float step_size;                 /* lr / (1 - beta1^t)               (torch/optim/adam.py) */
  float inv_bc2_sqrt;              /* 1 / sqrt(1 - beta2^t)                               */
} pert_adam_hparams;

/* Packed layout for (kind, L, N, K1, n_libs). */
int pert_make_layout(int32_t L, int32_t N, int32_t K1, int32_t n_libs, pert_layout* out);

/* Workspace element counts for cell_part (float), bin_part (float), blk_part (double),
 * cellblk_part (double) at bins_per_tile (0 = default).  cellblk_part must be
 * zero-initialised once: its last element holds pert_finalize's arrival counter, which
 * every finalize launch leaves at zero again. */
int pert_workspace_sizes(int32_t kind, int32_t L, int32_t N, int32_t K1, int32_t n_libs,
                         int32_t bins_per_tile, int64_t* n_cell_part, int64_t* n_bin_part,
                         int64_t* n_blk_part, int64_t* n_cellblk_part);

/* Bins per workgroup tile for the enumerated pass of this shard on the current device:
 * the tile length in [8, 64] whose grid (ldn/64 cell tiles x ceil(L/LT) bin tiles) best
 * fills whole rounds of the device's resident wave slots (occupancy queried for the
 * kernel instance and its LDS at that length), so a small shard does not end on a
 * partly filled last round.  Written to *out; steps 2/3 only (step 1 uses the default). */
int pert_auto_bins_per_tile(const pert_problem* prob, int32_t variant, int32_t* out);

/* Enumerated (steps 2/3) pass over every (bin, cell) of the shard.
 * Replaces the JitTraceEnum_ELBO forward + autograd backward of pert_model.py:801 / :868,
 * and with PERT_MODE_STEP the pi part of the Adam update; with PERT_MODE_DECODE it is
 * infer_discrete(temperature=0) of :820-827 / :886-893. */
int pert_enum_pass(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                   int32_t mode, hipStream_t stream);

/* One whole SVI step of steps 2/3 as ONE launch (variant 3 only): the PERT_MODE_STEP pass
 * with pert_finalize's reductions folded in -- the last bin tile of each cell tile to finish
 * reduces that tile's per-cell partials and runs Adam on its cells' u / betas / tau, the last
 * cell tile of each bin tile reduces that tile's rho partials, and the last of those adds
 * the global sums into grad_shared (loss in slot n_shared).  update_shared != 0 (a single
 * rank): the same launch also records the loss for the device loop and runs Adam on the
 * shared block.  update_shared == 0 (several ranks): all-reduce grad_shared, then
 * pert_adam_shared().  Uses the arrival counters at the end of cellblk_part (sized by
 * pert_workspace_sizes, zero-initialised once, re-armed by every launch).
 * Replaces svi.step() of pert_model.py:801 / :868 with the same update. */
int pert_enum_step(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                   int32_t update_shared, hipStream_t stream);

/* Adam on the shared block [0, n_shared) only (after the all-reduce of a pert_enum_step with
 * update_shared == 0), plus the device loop's loss record / stopping rule. */
int pert_adam_shared(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                     hipStream_t stream);

/* Observed (step 1) pass: JitTrace_ELBO forward + backward of pert_model.py:743.  In pair
 * mode (rep_obs == NULL, see the layouts above) one lane evaluates both copies of a G1/2 cell
 * from one load of its reads and CN (bins_per_tile up to 128). */
int pert_obs_pass(const pert_problem* prob, pert_state* st, hipStream_t stream);

/* Reductions of the pass partials + priors of the non-enumerated sites (pert_model.py:553-603)
 * -> grad_cell (local) and grad_shared (local partial sums incl. the loss in slot n_shared).
 * One launch: its last workgroup to finish adds the global sums. */
int pert_finalize(const pert_problem* prob, pert_state* st, hipStream_t stream);
/* pert_finalize split in two for a sharded step, so the shared block's all-reduce overlaps the
 * per-cell work: _shared writes grad_shared (local sums and loss) from the bin partials, the
 * pass's ELBO / d/da partials and the priors' terms (parameters only); _cells writes grad_cell
 * from each cell's partial rows and the u / beta / tau priors.  Together they write exactly
 * what pert_finalize writes; pert_adam follows both. */
int pert_finalize_shared(const pert_problem* prob, pert_state* st, hipStream_t stream);
int pert_finalize_cells(const pert_problem* prob, pert_state* st, hipStream_t stream);

/* Adam (torch.optim.Adam semantics, betas (0.8, 0.99)) on the packed params with
 * grad_shared (already all-reduced) and grad_cell. */
int pert_adam(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
              hipStream_t stream);

/* n whole SVI steps of a single-rank fit queued in one call (no all-reduce between the
 * reductions and Adam, so one rank only): for i < n the step of loop iteration iter0 + i
 * (st->step, the device loop's record index) with Adam hyper-parameters hp and
 * hp->step_size = step_size[i], hp->inv_bc2_sqrt = inv_bc2_sqrt[i] (host arrays the caller
 * computes for Adam steps t as torch.optim.Adam does: lr / (1 - beta1^t), 1 / sqrt(1 - beta2^t)).
 * Each step is pert_enum_step(update_shared = 1) when one_launch (steps 2/3, variant 3), else
 * pert_enum_pass(PERT_MODE_STEP) or pert_obs_pass, then pert_finalize and pert_adam.  With the
 * device loop armed (loop_ctl), the steps after the stopping one are no-ops.  pass_events
 * (NULL, or 2n caller-created events, NULL entries skipped): events[2i] / events[2i+1] are
 * recorded on the stream around step i's pass launch (the one launch of a one_launch step).  The call
 * only queues launches (a few microseconds each), so a binding may release its interpreter
 * lock around it.  Replaces n iterations of the svi.step loop of pert_model.py:742-758 /
 * :800-816 / :867-883 (the loss record and stopping rule stay on the device). */
int pert_svi_steps(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                   const float* step_size, const float* inv_bc2_sqrt, int32_t iter0, int32_t n,
                   int32_t one_launch, hipEvent_t* pass_events, hipStream_t stream);

/* A whole single-rank SVI fit with the device loop armed (st->loop_ctl / loop_rec set): up to
 * n_iter iterations queued in chunks of `chunk` (pert_svi_steps, step_size / inv_bc2_sqrt hold
 * all n_iter entries), each chunk followed by a copy of its loss records into host_rec (pinned
 * host memory, [n_iter][2] doubles) and an event; at most `depth` chunks are in flight, and
 * queueing ends once a copied record shows the stop.  pass_events: NULL, or 2 n_iter
 * caller-created events (NULL entries skipped) recorded around iteration i's pass as in
 * pert_svi_steps.  Returns after the stream has drained,
 * with *n_launched = the iterations queued (loop_ctl[0] holds the stopping iteration).  One
 * call per fit, so a binding that releases its interpreter lock around it leaves the host
 * thread free for the rest of the program for the whole fit.  Replaces the loop of
 * pert_model.py:742-758 / :800-816 / :867-883. */
int pert_svi_run(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                 const float* step_size, const float* inv_bc2_sqrt, int32_t n_iter, int32_t chunk,
                 int32_t depth, int32_t one_launch, hipEvent_t* pass_events, double* host_rec,
                 int32_t* n_launched, hipStream_t stream);

/* ---- Sharded fits: cells split over ranks, one process per GPU.
 * The shared block's gradient [0, n_shared) and the loss (slot n_shared) are summed across
 * the ranks once per SVI step, between the reductions and Adam.  A pert_comm is an RCCL
 * communicator over the fit's ranks (xGMI) -- or, for ranks sharing a GPU (which RCCL
 * refuses; tests), a host-staged sum through POSIX shared memory -- and the library queues
 * that all-reduce itself on the fit's stream, so a whole sharded fit is one C call like a
 * single-rank one.  Failure is bounded: a rank whose loop fails raises the node's abort word
 * (and aborts its RCCL communicator), and a rank waiting on its stream polls that word, RCCL's
 * async error and a deadline instead of blocking; the loop then returns PERT_E_COMM_ABORTED /
 * PERT_E_COMM_TIMEOUT / RCCL's error on every rank.  A comm is not usable after a failure. */
typedef struct pert_comm pert_comm;

/* dlopen RCCL from rccl_path (the copy the process already uses -- torch's) and resolve
 * ncclGetUniqueId / ncclCommInitRank / ncclAllReduce / ncclCommDestroy / ncclCommAbort /
 * ncclCommGetAsyncError.  Once per process. */
int pert_comm_load(const char* rccl_path);
/* ncclGetUniqueId into id (n = 128 bytes), on one rank; the caller broadcasts it. */
int pert_comm_unique_id(uint8_t* id, int32_t n);
/* ncclCommInitRank on the current device (collective: returns once every rank has called). */
int pert_comm_init(const uint8_t* id, int32_t n, int32_t world, int32_t rank, pert_comm** out);
/* The host-staged communicator: every rank of one node calls with the same POSIX shm name
 * ("/..."; the segment is unlinked once all ranks have mapped it) and max_n >= the longest
 * all-reduce; returns once every rank has attached or after timeout_s (PERT_E_COMM_TIMEOUT).
 * Each all-reduce is a copy to pinned memory, a host function summing the ranks' blocks in
 * rank order (identical bits on every rank) and a copy back, all queued on the stream. */
int pert_comm_init_host(const char* name, int32_t world, int32_t rank, int64_t max_n, double timeout_s,
                        pert_comm** out);
/* The deadline of every wait (seconds, default 600) and, for an RCCL communicator, a
 * node-local abort word: POSIX shm `abort_name` mapped collectively like pert_comm_init_host's
 * segment (NULL: the word is this process's own, peers then stop by the deadline). */
int pert_comm_set_watchdog(pert_comm* comm, const char* abort_name, double timeout_s);
/* Raise the abort word with `code` and, RCCL, abort the communicator (its queued collectives
 * return).  pert_svi_run_sharded calls it on any failure of its rank. */
int pert_comm_abort(pert_comm* comm, int32_t code);
/* PERT_OK, or the first failure seen by this rank (its own, or a peer's abort). */
int pert_comm_status(pert_comm* comm);
/* Wait for `ev` (recorded on the fit's stream) polling the abort word, RCCL's async error and
 * the deadline; on failure aborts the comm and returns the failure.  eager: poll without
 * sleeping (a wait whose end the caller's latency includes).  comm == NULL: hipEventSynchronize,
 * or with eager a poll. */
int pert_comm_wait_event(pert_comm* comm, hipEvent_t ev, int32_t eager);
/* Test hook: this rank's all-reduce call number `at_call` (0-based, -1 = never) fails at
 * queue time with PERT_E_COMM_FAULT, as a rank's launch failure would. */
int pert_comm_inject_fault(pert_comm* comm, int64_t at_call);
/* overlap (default 0, measured slower on ROCm 7.2: DESIGN.md section 6): pert_svi_run_sharded's
 * three-launch step runs split -- pert_finalize_shared,
 * the all-reduce on the comm's side stream (pert_comm_allreduce_async) while the fit's stream runs
 * pert_finalize_cells, then pert_comm_join + pert_adam; 0: pert_finalize, the all-reduce,
 * pert_adam on one stream.  delay_us > 0 (measurement only): every all-reduce also
 * runs a kernel spinning that long on its stream, a stand-in for an 8-rank ring's latency. */
int pert_comm_set_options(pert_comm* comm, int32_t overlap, double delay_us);
int pert_comm_overlap(const pert_comm* comm);
/* The all-reduce queued on the comm's side stream after the work already queued on `stream`
 * (overlap 0: on `stream` itself); pert_comm_join makes `stream` wait for it. */
int pert_comm_allreduce_async(pert_comm* comm, const double* send, double* recv, int64_t n, hipStream_t stream);
int pert_comm_join(pert_comm* comm, hipStream_t stream);
int pert_comm_destroy(pert_comm* comm);
/* recv = sum over ranks of send (fp64, n elements; send == recv allowed), queued on stream. */
int pert_comm_allreduce_sum_f64(pert_comm* comm, const double* send, double* recv, int64_t n,
                                hipStream_t stream);

/* pert_svi_steps / pert_svi_run of one rank of a sharded fit: each step's reductions write
 * this shard's shared-block sums to grad_local ([n_shared + 1] doubles), pert_comm_allreduce_sum_f64
 * sums them over the ranks into st->grad_shared, then Adam runs on the summed block
 * (pert_enum_step(update_shared = 0) + all-reduce + pert_adam_shared when one_launch; else
 * pass, pert_finalize, all-reduce, pert_adam).  Every rank stops after the same iteration
 * (the loss the rule tests is the all-reduced one) and queues the same number of
 * all-reduces.  Replaces the svi_s.step() loop of pert_model.py:800-816 on a cell shard. */
int pert_svi_steps_sharded(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                           const float* step_size, const float* inv_bc2_sqrt, int32_t iter0, int32_t n,
                           int32_t one_launch, pert_comm* comm, double* grad_local,
                           hipEvent_t* pass_events, hipStream_t stream);
int pert_svi_run_sharded(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                         const float* step_size, const float* inv_bc2_sqrt, int32_t n_iter, int32_t chunk,
                         int32_t depth, int32_t one_launch, pert_comm* comm, double* grad_local,
                         hipEvent_t* pass_events, double* host_rec, int32_t* n_launched, hipStream_t stream);

/* Diagnostic (bench.py): the HBM streams of pert_enum_pass(PERT_MODE_STEP) -- x, eta code,
 * z/m/v read and written back unchanged, same grid and tile length -- with no arithmetic.
 * Its duration is the access pattern's HBM ceiling on the running device; the state is
 * left bit-identical.  Steps 2/3 shards only. */
int pert_stream_ceiling(const pert_problem* prob, pert_state* st, hipStream_t stream);

/* tau initialiser (guess_times, pert_model.py:426-457): the batched pass of
 * manhattan_binarization (:364-423) for every cell in ONE launch, in fp64 -- standardisation,
 * GaussianMixture(n_components=2, random_state=0) (k-means++ and Lloyd initialisation, then EM),
 * the levels (GMM means, or percentiles chosen by the skew), the 100-threshold Manhattan scan --
 * twice per cell: run 0 breaks exact ties on a k-means decision towards centre 1, run 1 towards
 * centre 0.  Decisions that fp32 rounding (the reference's arithmetic) could flip are reported
 * in flags, so the caller recomputes those cells exactly (tau_init.exact_fractions). */
typedef struct {
  int32_t first;                   /* k-means++ first centre index (RandomState(0) draw) */
  int32_t lloyd_max_iter;          /* 300 (KMeans default) */
  int32_t em_max_iter;             /* 100 (GaussianMixture default) */
  int32_t q_lo[5], q_hi[5];        /* np.percentile 'linear' at q = .05 .25 .5 .75 .95: floor(q (L-1)), +1 (<= L-1) */
  int32_t pad_;
  double q_t[5];                   /* q (L-1) - floor(q (L-1)) */
  double u[2];                     /* the two local-trial uniforms of k-means++ */
  double tie;                      /* relative width of an exact tie on a k-means decision */
  double pp_margin;                /* k-means++ draw / choice margin, relative to the potential */
  double fragile;                  /* Lloyd shift-vs-tol margin, relative to tol */
  double em_margin;                /* EM |lower-bound change| vs tol margin, absolute */
  double em_tol;                   /* 1e-3 */
  double reg_covar;                /* 1e-6 */
  double mean_gap;                 /* 0.7  (MEAN_GAP_THRESH) */
  double early_skew, late_skew;    /* 0.2, -0.2 */
  double fragile_abs;              /* margin of the mean-gap / skew thresholds, absolute */
  double level_margin;             /* relative rounding budget of the scan levels (1e-6 sqrt(L)) */
  double eps32;                    /* float32 eps: the reference's summation noise in the scan */
} pert_tau_params;

/* norm: float [N][L] CN-normalised reads, one contiguous row per cell (device).
 * Outputs (device), per run r (0: ties to centre 1, 1: ties to centre 0) and cell n:
 *   labels  int8 [2][N][L]  final k-means labels (1 = centre 1)
 *   scratch int8 [2][N][L]  workspace
 *   means   double [2][N][2] GMM means
 *   flags   int32 [2][N]    bit 0: a Lloyd / EM stopping decision or the mean-gap / skew test
 *                           within its margin; bit 1: a k-means++ draw within its margin whose
 *                           alternatives end in other labels; bit 2: the scan's minimum within
 *                           its rounding slack of another threshold's
 *   frac    double [2][N]   replicated fraction (the reference's t_init where no flag is set)
 *   minor   double [2][N]   points within the levels' rounding budget of the chosen threshold */
int pert_tau_binarize(int32_t L, int32_t N, const float* norm, const pert_tau_params* p,
                      int8_t* labels, int8_t* scratch, double* means, int32_t* flags, double* frac,
                      double* minor, hipStream_t stream);

/* Test-only entry points: the per-(bin, cell) arithmetic of pert_math.h evaluated on
 * the host (no GPU needed) or on the device, for the parity suite.  Not used by any
 * product path. */
int pert_selftest_nb_lgdiff_host(int64_t n, const float* d, const float* x, float* lam, float* psi);
int pert_selftest_nb_lgdiff_device(int64_t n, const float* d, const float* x, float* lam, float* psi,
                                   hipStream_t stream);
int pert_selftest_enum_cellbin_host(int32_t P, int64_t n, const float* x, const float* em1,
                                    const float* S1, const float* z, float log1m_lam,
                                    const float* D, const float* phi, float* E, float* dirv,
                                    float* gD, float* gt, float* gz, int32_t* argmax);
/* The three-wave pass's per-element arithmetic (enum_online + the tail's logit gradient with
 * the argmax logit in jmax form) on the host: E and d(E + dirv)/dz. */
int pert_selftest_enum_online_host(int32_t P, int64_t n, const float* x, const float* em1,
                                   const float* S1, const float* z, float log1m_lam, const float* D,
                                   const float* phi, float* E, float* gz);

const char* pert_version(void);

#ifdef __cplusplus
}
#endif

#endif /* PERT_HIP_H */
