/*
 * gmt/engine.h — C ABI of the native Jacobi engine (libgmt_engine.so).
 *
 * The Python package drives the flagship benchmark through this ABI
 * (gpu_mpi_tests_amd/engine.py): torch.distributed does the rendezvous and
 * broadcasts a 128-byte id, then every step runs in C++ (hipGraph replay of
 * halo exchange + sweeps) with no Python on the critical path.  Transports:
 *   RCCL  one rank per GPU, xGMI; the id is an RCCL unique id;
 *   IPC   several ranks per GPU allowed (GPU oversubscription, the
 *         reference's mpi_daxpy.cc:43-54 mode) or one per GPU; HIP IPC
 *         mappings traded once over a Unix-socket mesh of the node named by
 *         the id (gmt_engine_control_id), one kernel launch per exchange;
 *   LOCAL one rank, no id.
 * No MPI in this library.
 */
#ifndef GMT_ENGINE_H
#define GMT_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum gmt_engine_transport { GMT_ENGINE_LOCAL = 0, GMT_ENGINE_RCCL = 1, GMT_ENGINE_IPC = 2 };

/* fills 128 bytes (an RCCL unique id); returns 0 or an error code */
int gmt_engine_unique_id(void* out128);
/* fills 128 bytes: the name of a socket control plane (GMT_ENGINE_IPC) */
int gmt_engine_control_id(void* out128);
/* Engine options (explicit fields; 0 = default everywhere). */
typedef struct gmt_engine_opts {
  int periodic; /* 1: periodic process grid, else Dirichlet (fixed ghost ring) */
  int overlap;  /* 0 off, 1 halo exchange overlapped with the core pass, 2 auto (time both once) */
  int graph;    /* 1: capture the per-parity passes into hipGraphs */
  int tsteps;   /* sweeps per fused pass and per halo exchange: 0 or 1 = single sweeps, else
                   2..GMT_TB_MAX_SWEEPS (odd values above 10 are rounded down to even) */
  int wg_waves; /* temporal-blocking kernel: waves per workgroup (0 = auto) */
  int seg_rows; /* temporal-blocking kernel: output rows per workgroup (0 = auto) */
  int exact;    /* -1 / 0: power-of-two scaled levels when the field bound allows (auto),
                   1: always the exact 1/4-per-level form */
  int init;     /* initial field: 0 = x^3 + y^2 on the global lattice, 1 = uniform [0, 1)
                   random (a hash of the global lattice point and `seed`) */
  int calibrate; /* 1: prepare() times every fused-pass size on the real share and the
                    planner uses those costs instead of the built-in table */
  int64_t seed;
  int push;     /* 1: inline halo exchange of the fused passes (JacobiConfig::push) */
} gmt_engine_opts;
/* id: 128 bytes (RCCL unique id / control id) or NULL (local); NULL on invalid options */
void* gmt_engine_jacobi_create(int64_t ny, int64_t nx, int py, int px, int rank, int world,
                               int transport, const void* ccl_id, const gmt_engine_opts* opts);
void gmt_engine_jacobi_destroy(void* h);
int gmt_engine_jacobi_run(void* h, int steps); /* enqueue `steps` steps */
int gmt_engine_jacobi_sync(void* h);
double gmt_engine_jacobi_residual(void* h);
int gmt_engine_jacobi_exchange(void* h); /* one blocking halo exchange */
/* out[16]: nx, ny, off_x, off_y, bytes_per_exchange, messages, graph, overlap, py, px, tsteps,
 * overlap_auto ns per pass with overlap, without (0 if not tuned), exact arithmetic in use,
 * band-first passes, inline halo exchange in use */
int gmt_engine_jacobi_info(void* h, int64_t* out);
/* The fused passes (sweeps per pass, in launch order) that run(steps) enqueues:
 * writes min(n, max) entries, returns n. */
int gmt_engine_jacobi_plan(void* h, int steps, int* out, int max);
/* The launch of the rank's one-rect K-sweep pass (gmt_jacobi5tb_plan's
 * info[6]); returns its error code. */
int gmt_engine_jacobi_tb_info(void* h, int K, int64_t* out);
/* Launch one pass of every pass type run(steps) will use, then restore the
 * initial field (first-launch costs stay out of a timed run). */
int gmt_engine_jacobi_prepare(void* h, int steps);
int gmt_engine_jacobi_copy_interior(void* h, double* host);
/* what: 0 = max |u| of the initial field (all ranks; drives the exactness
 * guard), 1 = measured ms of a full tsteps pass (0 before a calibrated
 * prepare), 2 = the built-in cost table's ms for that pass on this share */
/* bitwise comparison of the current interiors of two engines of the same
 * problem and process grid (collective): out[0] = max |diff| over ranks,
 * out[1] = elements whose bits differ, summed over ranks */
int gmt_engine_jacobi_compare(void* a, void* b, double* out);
/* gmt::plan_pass_sequence on given costs (cost[0..ks], ms per K-sweep pass):
 * the sweeps per pass, written to out[0..max); returns the plan length */
int gmt_engine_plan_from_costs(int k, int ks, const double* cost, int measured, int* out, int max);
/* reset != 0: zero the fused passes' clock record (stream ordered); else
 * out[3] = {shader MHz, samples, seconds sampled} since the last reset */
int gmt_engine_jacobi_clock(void* h, int reset, double* out);
double gmt_engine_jacobi_stat(void* h, int what);
const char* gmt_engine_backend(void);

/* A bare communicator on the same transports, for device collectives outside
 * the engine (bench.py's DAXPY partial-sum all-reduce, BASELINE config 3).
 * allreduce: in-place sum of n doubles in device memory, ordered on `stream`,
 * complete on return. */
void* gmt_engine_comm_create(int rank, int world, int transport, const void* id);
int gmt_engine_comm_allreduce_sum(void* h, double* buf, int64_t n, void* stream);
const char* gmt_engine_comm_name(void* h);
void gmt_engine_comm_destroy(void* h);
/* Hang watchdog (gmt/watchdog.hpp): armed by the first engine entry point
 * when GMT_TIMEOUT=<seconds> is set; the process exits with status 124 and a
 * "GMT WATCHDOG: rank R ... last phase '<phase>'" line when no phase mark
 * arrives for that long.  A caller marks progress of its own phases here. */
void gmt_engine_watchdog_kick(const char* phase);
double gmt_engine_watchdog_timeout(void); /* 0 when not armed */
/* Last words: when the watchdog fires, write `json` (an object) to stdout with
 * a "watchdog" field naming the stall and exit with `code` instead of 124; ""
 * exits with `code` silently; NULL restores the default. */
void gmt_engine_watchdog_epitaph(const char* json, int code);

/* The reference's halo-exchange benchmark (mpi_stencil2d_gt test_deriv for
 * dim 0 and dim 1, then test_sum), n_local x n_other per rank, 2 ghosts,
 * non-periodic 1-D slabs, on the RCCL or IPC transport (local for world == 1).
 * out[18]: per dim d (6 values at 6*d): exchange seconds median, mean, min,
 * max, bytes sent per exchange, this rank's err_norm; out[12] = all-reduce
 * (1024 doubles in place) median seconds, out[13] = its max relative error;
 * out[14 + d] = norm of the analytic derivative over this rank's output;
 * out[16 + d] = ghost cells found wrong after some exchange (check != 0: the
 * ghost rows are compared with the analytic field after EVERY exchange,
 * gmt/deriv.hpp; -1 without check). */
int gmt_engine_deriv_bench(int64_t n_local, int64_t n_other, int n_iter, int n_warmup, int rank,
                           int world, int transport, const void* ccl_id, double* out, int check);

#ifdef __cplusplus
}
#endif
#endif /* GMT_ENGINE_H */
