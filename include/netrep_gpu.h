/* netrep_gpu.h -- C ABI of the MI355X NetRep permutation engine.
 *
 * Plain pointers and sizes only; no C++ exceptions cross this boundary. All
 * matrices are R column-major fp64: A(i,j) at i + j*nrow. Every function
 * returns NR_OK (0) or an NR_ERR_* code; nr_last_error() has the message.
 *
 * Two layers:
 *  1. Engine layer (nr_*): one context per GPU holding ONE dataset resident
 *     in HBM, as the reference holds one dataset in RAM at a time
 *     (R/modulePreservation.R:553-620). It replaces the std::thread pool of
 *     calculateNulls (src/permutations.cpp:39-105, :335-380;
 *     src/permutationsNoData.cpp:35-89, :305-339) with batched device
 *     launches, and the Armadillo/LAPACK statistics of src/netStats.cpp with
 *     HIP kernels.
 *  2. Reference-interface layer (netrep_*): the eight Rcpp entry points of
 *     src/RcppExports.cpp:131-146 with the same argument meaning, taking
 *     names as C strings. An Rcpp glue unpacks SEXPs and
 *     calls these one-for-one.
 */
#ifndef NETREP_GPU_H
#define NETREP_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NR_OK 0
#define NR_ERR_HIP 1          /* HIP runtime / launch failure */
#define NR_ERR_INVALID 2      /* bad argument, shape or missing prerequisite */
#define NR_ERR_OOM 3          /* device allocation failed */
#define NR_ERR_UNSUPPORTED 4  /* size beyond an engine limit (n_nodes >= 2^31); modules of any
                                 size and any sample count are accepted, as svd_econ accepts any
                                 S x k block (src/netStats.cpp:217-280): Lanczos dimensions beyond
                                 the LDS vectors keep their vectors in device scratch */
#define NR_ERR_CANCELLED 5    /* nr_cancel() was called during a run */
#define NR_ERR_NONFINITE 6    /* CheckFinite failure (src/checkFinite.cpp:25-27) */

#define NR_HOST 0
#define NR_DEVICE 1

/* Statistic slots in the nulls cube (src/permutations.cpp:95-101, :174-177). */
#define NR_NSTAT_DATA 7
#define NR_NSTAT_NODATA 4

typedef struct nr_ctx nr_ctx;

/* ---- engine layer ------------------------------------------------------ */

int nr_device_count(int* count);
int nr_ctx_create(int device, nr_ctx** out);
void nr_ctx_destroy(nr_ctx* ctx);
/* Message of the last failing call on ctx (ctx == NULL: last nr_ctx_create failure). */
const char* nr_last_error(const nr_ctx* ctx);

/* Make one dataset resident: corr, net (n_nodes x n_nodes) and optional data
 * (n_samples x n_nodes, scaled as by Scale, src/scale.cpp:14-25; NULL for the
 * network-only path). `where` = NR_HOST or NR_DEVICE (device pointers, e.g.
 * after an RCCL broadcast). Replaces the previous dataset. The matrices are
 * stored interleaved as {corr(i,j), net(i,j)} pairs so one 16-byte read serves
 * CorrVector (src/netStats.cpp:196-201) and WeightedDegree (:135). */
int nr_set_dataset(nr_ctx* ctx, const double* corr, const double* net,
                   const double* data, int64_t n_nodes, int64_t n_samples, int where);
/* The same with flags: NR_SCALE_DATA = `data` is unscaled and is scaled on
 * the device (Scale, src/scale.cpp:14-25) on its way into HBM (NetProps,
 * src/properties.cpp:49). corr == net (same pointer): the matrix crosses
 * PCIe once and fills both halves of the pairs. */
#define NR_SCALE_DATA 1
int nr_set_dataset_ex(nr_ctx* ctx, const double* corr, const double* net,
                      const double* data, int64_t n_nodes, int64_t n_samples, int where, int flags);
/* Drop the resident dataset (and modules / null pool bound to it); the
 * context keeps its streams and scratch for the next dataset. */
int nr_clear_dataset(nr_ctx* ctx);

/* disk.matrix files straight to HBM (R/disk-matrix-class.R:175-182 reads them
 * back with readRDS): numeric matrices serialised by saveRDS (gzip or
 * uncompressed, XDR format 2/3) or objects of a save() archive (`*_object`,
 * NULL: the first numeric matrix). The payload is read straight into pinned
 * buffers and converted from big-endian on the device; `data` (samples x
 * nodes, NULL for the network-only path) is scaled there as Scale does
 * (src/scale.cpp:14-25) when scale_data != 0. The network file's column names
 * become the dataset's node names (nr_dataset_colnames). */
int nr_set_dataset_files(nr_ctx* ctx, const char* corr_path, const char* net_path, const char* data_path,
                         const char* corr_object, const char* net_object, const char* data_object,
                         int scale_data);
int nr_dataset_shape(const nr_ctx* ctx, int64_t* n_nodes, int64_t* n_samples);
/* NUL-separated node names of a dataset loaded from files; *needed = bytes
 * (written only when cap >= *needed). */
int nr_dataset_colnames(const nr_ctx* ctx, char* buf, int64_t cap, int64_t* needed);

/* Make src's resident dataset resident in dst too, device to device (over
 * xGMI when the contexts are on different GPUs): the host matrices cross PCIe
 * once, to the first GPU, and fan out from there. */
int nr_copy_dataset(nr_ctx* dst, const nr_ctx* src);
/* ctxs[0]'s resident dataset to ctxs[1..n): the broadcast of SURVEY.md 8e as
 * a scatter + all-gather of peer copies over the full xGMI mesh (each
 * destination receives one piece from the source and the other n - 2 pieces
 * from the destinations that received them; every link carries 1/(n-1) of
 * the bytes per phase). Contexts must be distinct; several may share a GPU.
 * Peer access is enabled per GPU pair; a pair without it is copied through
 * host memory by the runtime (slower, still correct) and counted by
 * nr_peer_staged_pairs. The calling thread's current device is restored. */
int nr_broadcast_dataset(nr_ctx* const* ctxs, int n);
/* Ordered GPU pairs found without peer access so far in this process. */
int nr_peer_staged_pairs(int* n);

/* 1 if corr and net of the resident dataset are exactly symmetric. */
int nr_dataset_symmetric(nr_ctx* ctx, int* symmetric);

/* 1 when the resident dataset carries the Gram table (the data block's
 * X^T X interleaved with the matrices, built by the first run or observed
 * call), else 0. Whether it is built depends on the shapes only (never on
 * free device memory): the packed-class modules (<= 320 nodes) must form one
 * packed-kernel launch (min(k, S) > 112, no module with more nodes than
 * samples), carry at least half the Gram work, and n_nodes <= 50,000; an
 * allocation failure then returns NR_ERR_OOM from the run / observed call
 * (DESIGN.md section 5.2). */
int nr_gram_table(nr_ctx* ctx, int* on);
/* Wall time in ms of the resident Gram table's build (X^T X on the matrix
 * cores + the widened layout, synchronised), 0 without a table. */
int nr_gram_table_ms(nr_ctx* ctx, double* ms);

/* CheckFinite (src/checkFinite.cpp:21-28) of the resident corr and net,
 * computed by nr_set_dataset's symmetry pass over the uploaded matrices (no
 * extra scan): 1 = every element finite. The caller raises the reference's
 * error ("matrices must not contain NaN/Inf", R/check-user-input.R:796-799). */
int nr_dataset_finite(nr_ctx* ctx, int* corr_finite, int* net_finite);

/* Module index sets (a4 of SURVEY.md 8) and discovery vectors (a15).
 *   n_rows      rows of the output cube = length of `modules`
 *   n_present   modules with >= 1 node in the test dataset (modsPresent,
 *               src/permutations.cpp:196-201), in `modules` order
 *   row_of      [n_present] output row of each present module
 *   node_off    [n_present+1] CSR offsets of module nodes
 *   test_idx    [node_off[n_present]] column of each node in the resident
 *               dataset (GetNodeIdx, src/utils.cpp:147-162); used for the
 *               observed statistics
 *   null_pos    [same] position of each node in the null pool (MakeNullMap
 *               nullMap, src/utils.cpp:108-136); may be NULL if no
 *               permutations will be run
 *   disc_corr   concatenated discovery CorrVector per module, k(k-1)/2 each
 *   disc_degree [nodes] discovery weighted degree (node order)
 *   disc_contrib[nodes] discovery node contribution, NULL for network-only */
int nr_set_modules(nr_ctx* ctx, int32_t n_rows, int32_t n_present,
                   const int32_t* row_of, const int64_t* node_off,
                   const int32_t* test_idx, const int32_t* null_pos,
                   const double* disc_corr, const double* disc_degree,
                   const double* disc_contrib);

/* The null pool nullIdx (MakeNullMap, src/utils.cpp:108-136): test columns. */
int nr_set_null_pool(nr_ctx* ctx, const int32_t* null_idx, int64_t n_null);

/* Observed statistics (src/permutations.cpp:246-285) into observed
 * [n_rows x n_stat], column-major (R matrix), NA_REAL for absent modules and
 * non-finite values (src/permutations.cpp:383-384). n_stat = 7 with data,
 * 4 without. */
int nr_observed(nr_ctx* ctx, double* observed);

/* The same, split so that it runs beside the permutations: nr_observed_async
 * enqueues the observed launch on the context's second stream (its own
 * scratch and work queue) and returns; nr_run / nr_run_device may follow at
 * once, and their first batch shares the GPU with it. nr_observed_wait
 * copies the statistics out (blocking). Any change of dataset, modules or
 * null pool in between waits for the launch and discards it (nr_observed_wait
 * then returns NR_ERR_INVALID). */
int nr_observed_async(nr_ctx* ctx);
int nr_observed_wait(nr_ctx* ctx, double* observed);

/* Null distributions for global permutations [perm_begin, perm_end).
 * pi == NULL: permutation p draws pi_p = keyed PRP(seed, p) (prp.h).
 * pi != NULL: explicit host table [(perm_end-perm_begin) x n_null] of
 *   null-pool permutations, pi[p][q] = source position (the exported
 *   shuffles of the reference, src/permutations.cpp:63). The table must hold
 *   exactly that many entries, each < n_null; an entry >= n_null is rejected
 *   with NR_ERR_INVALID before anything runs (device tables are checked by a
 *   device scan). Module nodes' null_pos (nr_set_modules) must be < n_null
 *   (NR_ERR_INVALID otherwise).
 * Cancellation: nr_cancel (any thread) stops the run in progress -- or the
 *   next one started on ctx -- between launches; it returns NR_ERR_CANCELLED
 *   with every slice not computed set to NA_real_ (the reference's
 *   interrupted workers leave their part of the NA-filled cube,
 *   src/permutations.cpp:375-384).
 * nulls receives (perm_end-perm_begin) slices of n_rows x n_stat, i.e. the
 * cube layout m + n_rows*s + n_rows*n_stat*p of src/permutations.cpp:55
 * starting at permutation perm_begin. Host pointer for nr_run, device pointer
 * for nr_run_device. */
int nr_run(nr_ctx* ctx, int64_t perm_begin, int64_t perm_end, uint64_t seed,
           const uint32_t* pi, double* nulls);
int nr_run_device(nr_ctx* ctx, int64_t perm_begin, int64_t perm_end,
                  uint64_t seed, const uint32_t* pi_device, double* nulls_device);

/* Host evaluation of the keyed null-pool permutation: out[p - perm_begin][q]
 * = pi_p(q) for q < n_null (no GPU needed). */
int nr_prp_table(uint64_t seed, int64_t perm_begin, int64_t perm_end,
                 int64_t n_null, uint32_t* out);

/* Export the index sets a run would use: test column of every module node of
 * permutations [perm_begin, perm_end), layout [perm][node] (CSR node order). */
int nr_export_indices(nr_ctx* ctx, int64_t perm_begin, int64_t perm_end,
                      uint64_t seed, int32_t* indices);

/* Per-module vectors for explicit index sets on the resident dataset
 * (IntermediateProperties src/discProps.cpp:92-122, NetProps
 * src/properties.cpp:152-185): corr_vec (k(k-1)/2 per module), degree (k),
 * avg_weight (one per module, AverageEdgeWeight src/netStats.cpp:154-162),
 * contribution (k), summary (n_samples per module) and coherence (one per
 * module, ModuleCoherence src/netStats.cpp:293-305). Any output may be NULL;
 * the last three need data. Node order = CSR order of idx. */
int nr_module_vectors(nr_ctx* ctx, int32_t n_mod, const int64_t* node_off,
                      const int32_t* idx, double* corr_vec, double* degree,
                      double* avg_weight, double* contribution, double* summary,
                      double* coherence);

/* Column scaling (Scale, src/scale.cpp:14-25) on the device. */
int nr_scale(nr_ctx* ctx, const double* data, int64_t n_samples,
             int64_t n_nodes, double* scaled);

/* CheckFinite (src/checkFinite.cpp:21-28): *all_finite = 1 or 0. */
int nr_check_finite(nr_ctx* ctx, const double* mat, int64_t n_elem, int* all_finite);

/* Progress (replaces MonitorProgress, src/thread-utils.cpp:49-82) and
 * cancellation (replaces the `interrupted` flag, src/permutations.cpp:362);
 * both are safe to call from another host thread during nr_run. */
int nr_progress(nr_ctx* ctx, int64_t* done, int64_t* total);
int nr_cancel(nr_ctx* ctx);

/* Tuning and measurement. */
int nr_set_batch(nr_ctx* ctx, int64_t perms_per_launch);
/* Host threads of the staging copies: the process-wide default for contexts
 * created afterwards (n <= 0: 8; capped at 16), and one context's own count.
 * The reference-interface calls set their contexts' count from n_cores and
 * never change the process default. */
int nr_set_host_threads(int n);
/* The process-wide default set by nr_set_host_threads (pooled contexts are
 * reset to it when a reference-interface call returns them). */
int nr_get_host_threads(void);
int nr_ctx_set_host_threads(nr_ctx* ctx, int n);
/* Host -> device bytes the library has copied since it was loaded (every
 * upload path counts): a caller can verify that resident data is not
 * uploaded again. */
int nr_h2d_bytes(int64_t* bytes);
int nr_set_timing(nr_ctx* ctx, int enable);
/* Accumulated device time (HIP events on the launch stream) per kernel:
 * kernel 0 = module network statistics, 1 = summary-profile statistics. */
int nr_get_timing(nr_ctx* ctx, int kernel, double* total_ms, int64_t* launches,
                  int64_t* items);
int nr_reset_timing(nr_ctx* ctx);
/* Summary-profile eigen-solver counters since the last nr_reset_timing:
 * items solved, Lanczos steps taken, items that reached the step cap, and
 * partial-reorthogonalisation passes performed. */
int nr_get_diagnostics(nr_ctx* ctx, int64_t* eig_items, int64_t* eig_steps,
                       int64_t* eig_cap_hits, int64_t* eig_reorths);
int nr_synchronize(nr_ctx* ctx);
/* Diagnostics: per-phase shader-cycle stamps of the summary-profile kernel,
 * summed over workgroups, 16 slots (0 index, 1 Gram, 2 Lanczos set-up,
 * 3 matvec, 4 three-term step + omega, 5 statistics, 6 q update, 7 Ritz
 * checks, 8 start column, 9 reorthogonalisation, 10 Ritz vector,
 * 11 node contributions, 12 Ritz coefficients, 13 a Ritz check's top
 * eigenvalue, 14 its residual (and the full-precision refinement where the
 * check may end the run; 7 keeps the rest of the check); 15 spare). Off by
 * default; a diagnostic build (make EXTRA=-DNR_STAMPS=1) records them; a run with stamps on
 * is a measurement run, not a timed one. */
int nr_set_stamps(nr_ctx* ctx, int enable);
int nr_get_stamps(nr_ctx* ctx, uint64_t* cycles);

/* Per-batch work buffers (column-sweep sets, profile-slot scratch, device
 * output and shuffle-table buffers): nr_release_scratch frees them (the next
 * run reallocates), nr_scratch_bytes reports what a context holds. The
 * reference-interface layer releases them whenever it pools a context. */
int nr_release_scratch(nr_ctx* ctx);
int nr_scratch_bytes(const nr_ctx* ctx, int64_t* bytes);
/* A context's own host-thread count (nr_ctx_set_host_threads). */
int nr_ctx_get_host_threads(const nr_ctx* ctx, int* n);

/* Test knobs, process-wide; neither changes a result. NR_DEBUG_SWEEP_MAX_OCC:
 * the column sweep's sub-batch bound in occurrences (value <= 0 restores the
 * default, 64M). NR_DEBUG_FAIL_SWEEP_ALLOC: the value-th column-sweep buffer
 * allocation from now fails with NR_ERR_OOM (0: off). */
#define NR_DEBUG_SWEEP_MAX_OCC 1
#define NR_DEBUG_FAIL_SWEEP_ALLOC 2
int nr_debug_set(int what, int64_t value);

/* ---- reference-interface layer ----------------------------------------- */
/* Names are arrays of NUL-terminated strings. moduleAssignments is the named
 * character vector as (node names, labels). Per-module discovery vectors are
 * given in `modules` order ([n_modules] pointers + lengths; NULL/0 for
 * modules absent from the test dataset). */

typedef struct netrep_disc_props {
  const double* const* degree;        /* [n_modules] */
  const int64_t* degree_len;
  const double* const* corr;
  const int64_t* corr_len;
  const double* const* contribution;  /* NULL for the network-only path */
  const int64_t* contribution_len;
} netrep_disc_props;

/* Interrupt hook: the replacement of checkInterrupt (src/interrupt.cpp:9-11)
 * as polled by MonitorProgress (src/thread-utils.cpp:49-82). While
 * netrep_PermutationProcedure runs, its calling thread polls fn(user) every
 * 100 ms (the engine works on other host threads); a non-zero return cancels
 * every GPU's run. The R glue installs a function that wraps
 * R_ToplevelExec(R_CheckUserInterrupt). NULL removes it.
 * Process-wide; set it before the call. */
typedef int (*netrep_interrupt_fn)(void* user);
void netrep_set_interrupt_hook(netrep_interrupt_fn fn, void* user);

/* Progress hook: the replacement of MonitorProgress's console output
 * (src/thread-utils.cpp:54-81: Rcpp::Rcout << endl, then "\r%5d% completed."
 * about once a second, then endl endl). While netrep_PermutationProcedure or
 * netrep_PermutationProcedureFiles runs with verbose != 0, the CALLING
 * thread -- the thread R called from, so the hook may write to
 * Rcpp::Rcout -- calls fn(event, done, total, user): NETREP_PROGRESS_BEGIN
 * once before the first permutation, NETREP_PROGRESS_UPDATE about once a
 * second and once more when the last permutation completes (done == total),
 * NETREP_PROGRESS_END once after the run (also after an interrupt).
 * netrep_format_progress renders an UPDATE exactly as the reference does.
 * The library itself never writes to stdout or stderr (R CMD check): with no
 * hook installed, verbose output is dropped. NULL removes the hook.
 * Process-wide; set it before the call. */
#define NETREP_PROGRESS_BEGIN 0
#define NETREP_PROGRESS_UPDATE 1
#define NETREP_PROGRESS_END 2
typedef void (*netrep_progress_fn)(int32_t event, int64_t done, int64_t total, void* user);
void netrep_set_progress_hook(netrep_progress_fn fn, void* user);
/* "\r%5d% completed." with the reference's rounding
 * ((unsigned)round((float)done / (float)total * 100), src/thread-utils.cpp:
 * 66-68) into buf (NUL-terminated, at most cap bytes); returns the length
 * written, or -1 if cap is too small. */
int netrep_format_progress(int64_t done, int64_t total, char* buf, int64_t cap);

/* PermutationProcedure (src/permutations.cpp:160-166) and
 * PermutationProcedureNoData (src/permutationsNoData.cpp:140-146, t_data =
 * NULL). nulls_out [n_modules x n_stat x n_perm], observed_out
 * [n_modules x n_stat], both column-major, NA-filled. `seed` keys the PRP;
 * `pi` (optional, [n_perm x n_null]) supplies explicit shuffles. n_cores
 * (nThreads of the reference, which sizes its worker pool) bounds the host
 * threads the call uses for its own work -- the pinned staging copies of the
 * test matrices (at most min(n_cores, 16) threads; n_cores <= 0: 8); the
 * permutations themselves run on the GPUs. NETREP_NUM_GPUS selects the GPU count
 * (NETREP_SHARE_DEVICE=1 lets several contexts share the visible GPUs, a test
 * mode for the sharded path on a one-GPU machine). The test matrices are
 * uploaded once, to the first GPU, and copied device to device to the others.
 * Interrupted (netrep_set_interrupt_hook): returns NR_ERR_CANCELLED with
 * observed_out complete and nulls_out holding every completed permutation,
 * NA_real_ elsewhere -- the partial cube the reference returns
 * (src/permutations.cpp:375-408). */
int netrep_PermutationProcedure(
    const netrep_disc_props* disc_props, const double* t_data,
    const double* t_corr, const double* t_net, int64_t n_samples,
    int64_t n_nodes, const char* const* t_names, const char* const* ma_names,
    const char* const* ma_labels, int64_t n_assign,
    const char* const* modules, int64_t n_modules, int64_t n_perm,
    int32_t n_cores, const char* null_hypothesis, int32_t verbose,
    uint64_t seed, const uint32_t* pi, double* nulls_out, double* observed_out);

/* Pipelining modulePreservation's loop over test datasets
 * (R/modulePreservation.R:553-620, one PermutationProcedure call per test
 * dataset): starts uploading the NEXT test dataset's matrices to GPU 0 in the
 * background (pinned, double-buffered chunks on the copy engine) and returns
 * at once: prefetch dataset t+1, then call netrep_PermutationProcedure on
 * dataset t, and the host->HBM copy of t+1 overlaps t's permutations. The
 * netrep_PermutationProcedure call naming the same three pointers and sizes
 * adopts the uploaded dataset instead of copying it again. At most two
 * prefetches are pending (the oldest is dropped beyond that); the arrays must
 * stay alive and unchanged until adopted or discarded. No reference
 * counterpart (the reference loads one test dataset at a time into RAM). */
int netrep_PrefetchTestDataset(const double* t_data, const double* t_corr, const double* t_net,
                               int64_t n_samples, int64_t n_nodes);
void netrep_DiscardPrefetch(void);

/* PermutationProcedure with the test dataset given as disk.matrix files
 * (R/disk-matrix-class.R; the R code would otherwise loadIntoRAM() them,
 * R/modulePreservation.R:553-620): the files go straight to GPU 0's HBM,
 * tData is scaled there, and the node names are the network file's column
 * names. The three files must agree on the node order: the correlation,
 * network and data files' column names (and the square matrices' row names)
 * must be identical where present, as R/check-user-input.R:757-771 requires
 * ("mismatch in node order between data, correlation, and network"). pi_len
 * is the number of entries in pi (n_perm x n_null, checked once the node
 * names -- hence n_null -- are known; -1: unchecked). Other arguments and
 * outputs as netrep_PermutationProcedure. */
int netrep_PermutationProcedureFiles(const netrep_disc_props* disc_props, const char* t_data_file,
                                     const char* t_corr_file, const char* t_net_file,
                                     const char* const* ma_names, const char* const* ma_labels,
                                     int64_t n_assign, const char* const* modules, int64_t n_modules,
                                     int64_t n_perm, int32_t n_cores, const char* null_hypothesis,
                                     int32_t verbose, uint64_t seed, const uint32_t* pi, int64_t pi_len,
                                     double* nulls_out, double* observed_out);

/* Host read of one numeric matrix from an RDS file or save() archive (the
 * same reader): dims always; values (column-major, native) into `out` when
 * non-NULL; NUL-separated column names into `colnames` when cap suffices
 * (*colnames_needed = bytes). No GPU involved. */
int netrep_ReadRDSMatrix(const char* path, const char* object, int64_t* nrow, int64_t* ncol, double* out,
                         char* colnames, int64_t colnames_cap, int64_t* colnames_needed);

/* IntermediateProperties[NoData] (src/discProps.cpp:44-48, :171-175).
 * Outputs per module in `modules` order, concatenated; lengths written to
 * *_len (0 for modules absent from the test node list). Buffers must hold
 * sum(k), sum(k(k-1)/2) and sum(k) doubles (k = module size in discovery). */
int netrep_IntermediateProperties(
    const double* d_data, const double* d_corr, const double* d_net,
    int64_t n_samples, int64_t n_nodes, const char* const* d_names,
    const char* const* t_node_names, int64_t n_t_nodes,
    const char* const* ma_names, const char* const* ma_labels,
    int64_t n_assign, const char* const* modules, int64_t n_modules,
    double* degree_out, int64_t* degree_len, double* corr_out,
    int64_t* corr_len, double* contribution_out, int64_t* contribution_len);

/* NetProps[NoData] (src/properties.cpp:41-44, :190-193). data is unscaled
 * (NetProps scales internally, :49). Per module (in `modules` order) with
 * k_all = all module nodes in moduleAssignments order: degree[k_all],
 * contribution[k_all], summary[n_samples], coherence, avg_weight; NA for
 * absent nodes (:133-139). *_len receive k_all per module. */
int netrep_NetProps(const double* data, const double* net, int64_t n_samples,
                    int64_t n_nodes, const char* const* node_names,
                    const char* const* ma_names, const char* const* ma_labels,
                    int64_t n_assign, const char* const* modules,
                    int64_t n_modules, double* degree_out,
                    double* contribution_out, double* summary_out,
                    double* coherence_out, double* avg_weight_out,
                    int64_t* k_all_out);

/* Scale (src/scale.cpp:38-45): the host matrix through the context's pinned
 * staging in ~16 MiB column chunks, scaled on the device, copied back. */
int netrep_Scale(const double* data, int64_t n_samples, int64_t n_nodes,
                 double* scaled_out);

/* CheckFinite (src/checkFinite.cpp:21-28): NR_ERR_NONFINITE with the
 * reference's message if any element is NA/NaN/Inf. */
int netrep_CheckFinite(const double* mat, int64_t nrow, int64_t ncol);

/* Residency across calls of the reference-interface layer (modulePreservation
 * calls IntermediateProperties and PermutationProcedure once per (discovery,
 * test) pair, R/modulePreservation.R:553-635; networkProperties calls NetProps
 * once per pair, R/networkProperties.R:295-302): the discovery dataset of
 * netrep_IntermediateProperties and the dataset of netrep_NetProps stay
 * resident in HBM while later calls name the same host arrays (same
 * pointers and shape, and the same fingerprint of every element, hashed on
 * the process-wide host threads of nr_set_host_threads -- a full pass over
 * the host arrays at memory bandwidth, the price of reuse; a sampled check
 * of 4,096 elements per array runs first, so a changed array skips the full
 * pass); contexts (streams) are pooled across calls, and a pooled context is
 * reset to the defaults (no dataset, no per-batch work buffers, no cancel
 * request, the process-wide host-thread count). A changed array
 * is uploaded again. netrep_ReleaseResident frees all of it (the R glue calls
 * it when modulePreservation / networkProperties return); a
 * netrep_PermutationProcedure call that runs out of device memory releases
 * the resident datasets and retries once before returning NR_ERR_OOM. */
void netrep_ReleaseResident(void);
/* The pooled contexts (idle between calls): how many, the device bytes of
 * per-batch work buffers they hold (0: released), and the range of their
 * host-thread counts (each equals nr_get_host_threads after a call). With
 * no pooled context the thread range is 0, 0. */
int netrep_PoolInfo(int64_t* n_pooled, int64_t* scratch_bytes, int32_t* host_threads_min,
                    int32_t* host_threads_max);

/* Last error of the reference-interface layer (thread-local). */
const char* netrep_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* NETREP_GPU_H */
