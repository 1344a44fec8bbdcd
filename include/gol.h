/*
 * gol.h -- C ABI of libgol, the MI355X-native generation-step engine.
 *
 * This is the drop-in boundary for the reference's hot path: the cell-actor
 * generation step of almendar/akka-game-of-life.  The reference has no FFI;
 * its "interface" is the Akka cell protocol.  Each entry point below names
 * the reference interface it replaces (paths relative to
 * src/main/scala/gameoflife/ of the reference).
 *
 * Conventions (DESIGN.md "Boundary"):
 *   - Plain C types only: POD structs, pointers and sizes.  No torch types.
 *   - Return 0 (GOL_OK) on success, a GOL_E* code otherwise; a per-context
 *     message is available from gol_last_error().  A JVM/ctypes shim maps a
 *     nonzero code to an exception, which is where the reference's supervisor
 *     Restart (BoardCreator.scala:42-45) would take over.
 *   - A context owns device memory on one GPU.  Host buffers belong to the
 *     caller.  A context is not re-entrant, but calls may arrive from any OS
 *     thread (actor dispatchers): every entry point re-binds its device.
 *   - There is no CPU fallback: a context can only be created on a HIP
 *     device; without one gol_create() fails with GOL_ENODEV.
 *
 * Host buffers (gol_load, gol_snapshot, checkpoints): bit-packed rows,
 * row = y, bit (x % 32) of 32-bit word (x / 32) is cell x (LSB first); words
 * per row = ceil(width / 32); bits at x >= width are zero.
 * Device layout (internal, a function of the geometry alone): the same rows,
 * except that tori whose rows hold an even number of words are kept
 * pair-interleaved (gol_device_layout) -- word 2k + j holds columns
 * 64k + 2b + j (bit b).  Two device planes (current / next) are swapped after
 * every pass.
 *
 * State hash (gol_hash, gol_step's per-generation hashes; DESIGN.md section
 * 5): a function of the cells alone -- the same board at the same epoch
 * hashes alike whatever the topology, layout, shard decomposition, pass
 * depth or environment.  Columns 64g .. 64g + 63 of row y form group g, with
 * canonical words E (bit b = cell 64g + 2b) and O (bit b = cell 64g + 2b + 1),
 * cells past the width dead; then
 *   hash = sum over (y, g) of (E A(y, 0) + O A(y, 1)) B(g)   (mod 2^64),
 *   A(y, 0) = ((t ^ (t >> 15)) << 1) | 1,  t = y * 0x9E3779B1 (mod 2^32),
 *   A(y, 1) = A(y, 0) + 0x6A09E666,  B(g) = murmur3 fmix32(g + 0x7F4A7C15) | 1.
 */
#ifndef GOL_H
#define GOL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 5): the state hash became a function of the cells alone (see the
 * header comment); the values of tori with an even word count are unchanged,
 * those of row-major boards (clipped, odd word counts) differ from version 1.
 * The entry points and structs are those of version 1. */
#define GOL_ABI_VERSION 2

/* Return codes. */
#define GOL_OK 0
#define GOL_EINVAL 1   /* bad argument / unsupported geometry               */
#define GOL_EHIP 2     /* HIP runtime error                                 */
#define GOL_ENOMEM 3   /* device or host allocation failed                  */
#define GOL_ECOMM 4    /* RCCL error / communicator not initialised         */
#define GOL_ESTATE 5   /* call not valid in the context's current state     */
#define GOL_ENODEV 6   /* no HIP device (no CPU fallback exists)            */

/* Topologies. */
#define GOL_TORUS 0        /* wrap in x and y (BASELINE.json configs 2-5)     */
#define GOL_REF_CLIPPED 1  /* reference geometry: (w+1)x(h+1) cells, neighbours
                              only from [0,w)x[0,h) (BoardCreator.scala:47-53,
                              package.scala:17-28)                            */

/* Life-like rules as (birth_mask, survive_mask): bit k set = the rule fires
 * at k live neighbours.  NextStateCellGathererActor.scala:42-44. */
#define GOL_RULE_LIFE_BIRTH 0x008u          /* B3/S23 (north_star)          */
#define GOL_RULE_LIFE_SURVIVE 0x00Cu
#define GOL_RULE_REF_LITERAL_BIRTH 0x000u   /* line 44 with a multiset count */
#define GOL_RULE_REF_LITERAL_SURVIVE 0x1F7u
#define GOL_RULE_REF_EFFECTIVE_BIRTH 0x000u /* line 42's Set collapse: the   */
#define GOL_RULE_REF_EFFECTIVE_SURVIVE 0x1FFu /* identity, what actually runs */

#define GOL_UNIQUE_ID_BYTES 128

typedef struct gol_ctx gol_ctx;

/* Board / shard description.  Replaces the BoardCreator constructor inputs
 * (boardSize, BoardCreator.scala:18; application.conf:29-35) plus the cell
 * placement (BoardCreator.scala:65-70): a context owns the row block
 * [row0, row0 + rows) of a width x height board. */
typedef struct gol_config {
    int64_t width;          /* cells per row (torus: multiple of 32), < 2^31  */
    int64_t height;         /* rows of the global board                       */
    int64_t row0;           /* first global row owned by this context         */
    int64_t rows;           /* rows owned (0 => height - row0)                */
    int32_t topology;       /* GOL_TORUS or GOL_REF_CLIPPED                   */
    uint32_t birth_mask;    /* 9-bit masks, see GOL_RULE_*                    */
    uint32_t survive_mask;
    int32_t device;         /* HIP device ordinal                             */
    int64_t vis_width;      /* REF_CLIPPED: visible columns (0 => width-1)    */
    int64_t vis_height;     /* REF_CLIPPED: visible rows    (0 => height-1)   */
} gol_config;

/* Create a shard context.  Replaces createAllInitialActors
 * (BoardCreator.scala:79-89) + CellActor construction (CellActor.scala:10,
 * 34: epochToState = Map(0 -> initialState)).  The board starts all dead at
 * epoch 0; fill it with gol_seed() or gol_load().
 * GOL_REF_CLIPPED boards on which some cell has no visible neighbour are
 * refused with GOL_EINVAL: the reference never completes a generation on them
 * (such a cell's gatherer has nobody to ask, so it never commits an epoch,
 * NextStateCellGathererActor.scala:26-27,39-58, and its neighbours' requests
 * for that epoch queue forever, CellActor.scala:75-76,92-94).  With the
 * default visible extents that is a board of size w = 0 or h = 0 (one cell
 * wide or tall) or w = h = 1 (2 x 2 cells). */
int gol_create(gol_ctx** out, const gol_config* cfg);

/* Free device memory and streams.  Replaces stopping the cell actors. */
void gol_destroy(gol_ctx* ctx);

/* Last error message of this context ("" if none); ctx may be NULL for the
 * process-wide last error (e.g. a failed gol_create). */
const char* gol_last_error(const gol_ctx* ctx);
const char* gol_strerror(int code);
int gol_abi_version(void);

/* Number of HIP devices visible to this process (0 on a CPU-only host). */
int gol_device_count(int* count);

/* Row-block decomposition used for sharding (DESIGN.md "Multi-GPU"): rank r
 * of n owns rows [row0, row0 + rows) of a board `height` rows tall.  Pure
 * host arithmetic.  Replaces the random placement of BoardCreator.scala:33-36. */
int gol_shard_rows(int64_t height, int rank, int nranks, int64_t* row0, int64_t* rows);

/* Device layout of a board (pure host arithmetic,
 * informational): *words_per_group = 2 when a torus row holds whole pairs of
 * 32-bit words (column 64g + 2b + j in bit b of word 2g + j), 1 (row-major:
 * column x in bit x % 32 of word x / 32) otherwise and on clipped boards.
 * Nothing at the boundary depends on it: host buffers are row-major and the
 * state hash is defined over the cells. */
int gol_device_layout(int32_t topology, int64_t width, int32_t* words_per_group);

/* Seed the shard with the counter-based splitmix64 board (Bernoulli(0.5)),
 * identical for any sharding; resets the epoch to 0.  Seeded stand-in for
 * BoardCreator.scala:23 (initialState = Random.nextBoolean() per cell). */
int gol_seed(gol_ctx* ctx, uint64_t seed);

/* Load the shard from host memory: `rows` x `host_pitch_words` packed words
 * (row 0 = global row row0).  Resets the epoch to 0.  Replaces the per-cell
 * initialState constructor argument (BoardCreator.scala:67-68). */
int gol_load(gol_ctx* ctx, const uint32_t* packed, int64_t host_pitch_words);

/* Advance `generations` generations.  Replaces one NextStep tick
 * (BoardCreator.scala:113-116) -> CurrentEpochMsg -> GetToNextEpoch ->
 * NextStateCellGathererActor gather/count/rule -> SetNewStateMsg commit
 * (CellActor.scala:63-91, NextStateCellGathererActor.scala:25-48), for every
 * cell of the shard at once.  If hashes_out is not NULL it receives, for each
 * generation, the shard's partial state hash (DESIGN.md "State hash"); the
 * global hash is the sum mod 2^64 of the shards' partials; hashes_out must
 * hold `generations` entries (gol_step_ex checks a capacity).  With a
 * communicator attached, G halo rows are exchanged over RCCL before every pass
 * of G generations.  Asynchronous when hashes_out is NULL (call gol_sync to
 * wait). */
int gol_step(gol_ctx* ctx, uint32_t generations, uint64_t* hashes_out);

/* gol_step with the capacity of hashes_out (entries): GOL_EINVAL, and no
 * generation advanced, when hashes_out is not NULL and holds fewer than
 * `generations` entries.  The form a JVM binding calls with a direct buffer's
 * capacity. */
int gol_step_ex(gol_ctx* ctx, uint32_t generations, uint64_t* hashes_out, size_t hashes_capacity);

/* Light-cone replay of a re-spawned shard, alone.  Replaces the reference's
 * re-born cell catching up from its neighbours' never-pruned histories
 * (BoardCreator.scala:138-154 re-deploys it, CellActor.scala:34,71-74,86 it
 * replays epoch by epoch from their answers).  ctx holds its rows at epoch e
 * (gol_restore of its own checkpoint); `above` holds the n = `generations`
 * rows just above row0 and `below` the n rows just below row0 + rows, as they
 * were at epoch e (global rows row0 - n .. row0 - 1 and row0 + rows ..
 * row0 + rows + n - 1, modulo the height on a torus; dead rows beyond a
 * clipped board's edge), row-major host rows `host_pitch_words` apart.  The
 * block n rows deeper on each side fixes the shard's rows for n generations,
 * so ctx advances n generations exactly as if its neighbours had been there,
 * while they stay where they are.  hashes_out (nullable, n entries) receives
 * the shard's per-generation partial hashes.  The context must not belong to
 * a group or ring yet (GOL_ESTATE). */
int gol_replay(gol_ctx* ctx, uint32_t generations, const uint32_t* above, const uint32_t* below,
               int64_t host_pitch_words, uint64_t* hashes_out);

/* Current epoch (CellActor.scala:39 myCurrentEpoch). */
int gol_epoch(const gol_ctx* ctx, uint64_t* epoch);

/* Block until all work queued on the context's streams is complete. */
int gol_sync(gol_ctx* ctx);

/* Partial state hash of the shard's current board. */
int gol_hash(gol_ctx* ctx, uint64_t* hash_out);

/* Copy the shard's current board to host: rows x host_pitch_words words.
 * Replaces the CellStateMsg stream to the LoggerActor
 * (CellActor.scala:89, LoggerActor.scala:30-46). */
int gol_snapshot(gol_ctx* ctx, uint32_t* packed_out, int64_t host_pitch_words);

/* Periodic snapshots without stalling the generation pipeline: the same copy
 * as gol_snapshot, started at the current epoch and finished in the
 * background while later gol_step calls run (LoggerActor's periodic board
 * dump, LoggerActor.scala:30-46, fed by one CellStateMsg per cell and epoch,
 * CellActor.scala:89).  The board is first copied on the device (one more
 * plane of HBM, allocated on first use), then to `packed_out` on a transfer
 * stream.  `packed_out` must stay valid and unread until gol_snapshot_wait
 * returns; page-locked memory (gol_host_alloc) keeps the call from blocking
 * on a staged copy.  One snapshot in flight per context (GOL_ESTATE). */
int gol_snapshot_async(gol_ctx* ctx, uint32_t* packed_out, int64_t host_pitch_words);

/* Wait for the snapshot started by gol_snapshot_async; *epoch_out (may be
 * NULL) receives the epoch the copy holds.  GOL_ESTATE if none is in flight. */
int gol_snapshot_wait(gol_ctx* ctx, uint64_t* epoch_out);

/* Non-blocking: *landed = 1 if the snapshot started by gol_snapshot_async
 * has reached the host buffer, 0 if it is still in flight (a JVM worker polls
 * this instead of blocking its actor thread; the fault path asks it of a lost
 * shard: a checkpoint that had not landed when the backend died never
 * existed).  GOL_ESTATE if none is in flight.  gol_snapshot_wait still ends
 * the snapshot. */
int gol_snapshot_query(gol_ctx* ctx, int* landed);

/* Page-locked host memory for snapshot / load buffers (the JVM side wraps it
 * in a direct ByteBuffer); free with gol_host_free. */
int gol_host_alloc(size_t bytes, void** out);
void gol_host_free(void* p);

/* State of one cell of the shard at the current epoch (0/1).  Replaces the
 * GetStateFromEpoch -> StateForEpoch exchange (CellActor.scala:71-77). */
int gol_get_cell(gol_ctx* ctx, int64_t x, int64_t y, int* state);

/* Shard checkpoint = {header with epoch + geometry, packed board}.  Replaces
 * the reference's recovery state (initialState kept by the frontend,
 * BoardCreator.scala:23,144, plus each cell's never-pruned history,
 * CellActor.scala:34,81) used when a cell is re-deployed
 * (BoardCreator.scala:138-154). */
int gol_checkpoint_bytes(const gol_ctx* ctx, size_t* bytes);
int gol_checkpoint(gol_ctx* ctx, void* host_out, size_t bytes);

/* gol_checkpoint in the background (the periodic checkpoint of the fault
 * path overlapping the generations after it): the header is written now, the
 * rows follow as with gol_snapshot_async; finish with gol_snapshot_wait.
 * GOL_ESTATE while a snapshot or checkpoint is in flight. */
int gol_checkpoint_async(gol_ctx* ctx, void* host_out, size_t bytes);
int gol_restore(gol_ctx* ctx, const void* host_in, size_t bytes);

/* Multi-GPU: RCCL communicator over the ring of row-block shards.  Replaces
 * the cross-backend neighbour messages (GetStateFromEpoch/StateForEpoch over
 * Akka remote, application.conf:11-17).  Rank 0 calls gol_comm_unique_id and
 * distributes the bytes; every rank then calls gol_comm_init.  A context
 * with a communicator always runs the ring schedule (interior rows || halo
 * send/recv, then boundary rows); with nranks = 1 the torus ring closes on
 * itself (send/recv to self), which runs the RCCL path on a single GPU. */
int gol_comm_unique_id(uint8_t id_out[GOL_UNIQUE_ID_BYTES]);
int gol_comm_init(gol_ctx* ctx, const uint8_t id[GOL_UNIQUE_ID_BYTES], int rank, int nranks);

/* Tear down the context's communicator (ncclCommAbort: safe with a dead
 * peer); gol_comm_init may then join a new ring.  The shard keeps its board
 * and epoch.  Used when a lost backend is re-spawned and the survivors rebuild
 * the ring around it (gameoflife/elastic.py). */
int gol_comm_abort(gol_ctx* ctx);

/* Test transport: join the in-process loopback ring `key` as rank/nranks
 * instead of an RCCL communicator.  Contexts of one process -- one host
 * thread each, as one process per GPU would be -- then run exactly the halo
 * exchange gol_step issues over RCCL (the same send / receive list in the
 * same order, matched per (sender, receiver) pair in FIFO order like
 * ncclSend / ncclRecv) as device copies, and gol_comm_allreduce_u64 sums over
 * them.  This runs the multi-rank schedule with several ranks on one GPU,
 * where RCCL refuses a second rank.  gol_comm_abort leaves the ring. */
int gol_comm_init_loopback(gol_ctx* ctx, const char* key, int rank, int nranks);

/* Sum-reduce `count` uint64 values (mod 2^64) across the communicator in
 * place (the per-generation hash reduction). */
int gol_comm_allreduce_u64(gol_ctx* ctx, uint64_t* values, uint32_t count);

/* In-process shard group: several shard contexts of one board, in row order
 * and covering it without gaps, possibly on different GPUs (or several on
 * one), stepped in lockstep with halo rows pulled by device-to-device copies
 * (the same interior / boundary schedule as an RCCL ring).  This is how one
 * surviving GPU hosts a re-spawned shard next to its own (the reference
 * re-deploys a dead cell on a random surviving node, BoardCreator.scala:138-154).
 * Destroying a member leaves a hole: gol_group_step then fails with
 * GOL_ESTATE until the group is rebuilt.  gol_group_destroy unlinks the
 * shards without destroying them.  hashes_out receives the global hash. */
typedef struct gol_group gol_group;
int gol_group_create(gol_group** out, gol_ctx* const* shards, int n);
int gol_group_step(gol_group* group, uint32_t generations, uint64_t* hashes_out);
/* gol_group_step that also returns every shard's per-generation partial
 * hashes: partials_out[k * generations + g] = shard k's partial of generation
 * g (hashes_out required).  The fault path keeps them to check a re-spawned
 * shard's replayed partials against the recorded global hashes. */
int gol_group_step_partials(gol_group* group, uint32_t generations, uint64_t* hashes_out, uint64_t* partials_out);
int gol_group_sync(gol_group* group);
const char* gol_group_last_error(const gol_group* group);
void gol_group_destroy(gol_group* group);

/* Kernel timing: when enabled, the dominant step-kernel launch of every pass
 * (the whole shard, or a sharded shard's interior rows) is bracketed by HIP
 * events on the stream it runs on.  gol_profile_read returns, since the last
 * reset, the summed duration (ms), the number of launches and the number of
 * generations those launches advanced (a pass may fuse several). */
int gol_profile_enable(gol_ctx* ctx, int enable);
int gol_profile_read(gol_ctx* ctx, double* total_ms, uint64_t* launches, uint64_t* generations);
int gol_profile_reset(gol_ctx* ctx);
/* Clock (GHz) the GPU held during the profiled launches since the last
 * reset, time-weighted: each launch's workgroups read their XCD's core-clock
 * and 100 MHz reference counters at start and end (0 if none recorded). */
int gol_profile_clock(gol_ctx* ctx, double* ghz);

/* Per-rank breakdown of the profiled passes of a sharded context (the cost
 * of the cross-backend exchange the reference carries as GetStateFromEpoch /
 * StateForEpoch messages, CellActor.scala:71-77,
 * NextStateCellGathererActor.scala:32-36).  Since the last
 * gol_profile_reset, with profiling enabled:
 *   kernel_ms / launches / generations: as gol_profile_read (the dominant
 *       launch: the whole shard, or a sharded shard's interior rows);
 *   exchange_ms / exchanges: the halo exchange of each sharded pass, timed by
 *       HIP events on the comm stream around the RCCL group (or loopback
 *       copies): from the moment the plane is final to the moment every send
 *       and receive of the pass has completed -- waiting for a late peer
 *       included;
 *   boundary_ms / boundary_launches: the boundary-row launches on the edge
 *       stream;
 *   halo_bytes_sent / halo_bytes_received: bytes posted to / expected from
 *       the ring's send and receive operations (counted whether or not
 *       profiling is enabled);
 *   clock_ghz: as gol_profile_clock;
 *   exchange_exposed_ms / pass_tail_ms: per pass, how long after the end of
 *       its interior launch the exchange (resp. the boundary launch) ended,
 *       0 if before, summed: the part of the exchange the interior did not
 *       hide, and the pass's whole critical path beyond the interior. */
typedef struct gol_profile_stats {
    double kernel_ms;
    uint64_t launches;
    uint64_t generations;
    double exchange_ms;
    uint64_t exchanges;
    double boundary_ms;
    uint64_t boundary_launches;
    uint64_t halo_bytes_sent;
    uint64_t halo_bytes_received;
    double clock_ghz;
    double exchange_exposed_ms;  /* sum over passes of how long the exchange ended after the interior launch (>= 0) */
    double pass_tail_ms;         /* ... and the boundary launch: the pass's critical path beyond the interior */
} gol_profile_stats;
int gol_profile_stats_read(gol_ctx* ctx, gol_profile_stats* out);

/* The runtime stack this process's libgol is bound to: the HIP runtime and
 * RCCL versions it calls and the files the dynamic linker resolved them to
 * (dladdr of a symbol of each), plus libgol's own path.  Host-only: needs no
 * device.  A JVM host and the Python tools report the same fields, so a
 * multi-rank run states which library stack it exercised. */
typedef struct gol_runtime_info {
    int32_t abi_version;
    int32_t hip_runtime_version;  /* hipRuntimeGetVersion (0 if it failed)  */
    int32_t hip_driver_version;   /* hipDriverGetVersion  (0 if it failed)  */
    int32_t rccl_version;         /* ncclGetVersion, e.g. 22707 = 2.27.7    */
    char hip_library[512];        /* path of the libamdhip64 in use         */
    char rccl_library[512];       /* path of the librccl in use             */
    char gol_library[512];        /* path of this libgol                    */
} gol_runtime_info;
int gol_runtime_info_get(gol_runtime_info* out);

/* Tuning knobs (results never depend on them); 0 selects the automatic
 * choice, which is also the default of a new context:
 *   band_rows       rows of output streamed by one wave;
 *   gens_per_pass   generations fused per HBM pass (temporal blocking, 1..12;
 *                   automatic: the pass planner, see gol_pass_plan);
 *   words_per_lane  32-bit words each lane owns per row (1, 2 or 4; must
 *                   divide the words of a row).
 * GOL_EINVAL for words_per_lane = 4 together with gens_per_pass > 7 on any
 * board but the B3/S23 torus: those kernel instances (generic rule masks,
 * clipped visibility) would spill registers to scratch and are not built
 * (the planner caps planned passes of such a tuning at 7). */
int gol_set_tuning(gol_ctx* ctx, int32_t band_rows, int32_t gens_per_pass, int32_t words_per_lane);

/* Diagnostic: the pass depths (generations fused per HBM pass) gol_step would
 * use to advance `generations` generations (at most 1024: gol_step plans per
 * chunk of 1024) with or without per-generation hashes, in launch order.
 * Writes at most `max` depths to `depths` and their number to `count`. */
int gol_pass_plan(gol_ctx* ctx, uint32_t generations, int32_t with_hashes, int32_t* depths, int32_t max,
                  int32_t* count);

/* Diagnostic: resident 64-lane waves per CU of the step kernel a pass of
 * `gens_per_pass` generations would launch with the context's current
 * tuning (occupancy API), and the strip width in words (a whole row for the
 * whole-row waves of a 4096-column B3/S23 torus at 10-generation passes). */
int gol_occupancy(gol_ctx* ctx, int32_t gens_per_pass, int32_t* waves_per_cu, int32_t* strip_words);

/* Diagnostic: runs a one-wave kernel exercising the cross-lane primitives the
 * step kernel relies on (DPP wave shifts, v_alignbit, scalar loads) and
 * writes 256 words to report (layout: gol_kernels.hip selftest_kernel). */
int gol_selftest(int device, uint32_t* report);

/* Diagnostics of the HIP status discipline.  A failing
 * HIP call leaves its status pending on the calling thread (hipGetLastError);
 * libgol takes every status it reports or logs off the thread, launches its
 * kernels with calls that return their own status, and absorbs what RCCL's
 * own HIP calls leave behind right after each RCCL call.  So after any libgol
 * entry point the thread has no pending HIP status that libgol produced.
 *   gol_diag_take_hip_error: the calling thread's pending HIP status (0: none),
 *                            taken off the thread (hipGetLastError).
 *   gol_diag_absorbed:       how many statuses RCCL calls left behind, and the
 *                            last one's description (`last` may be NULL). */
int gol_diag_take_hip_error(int* code);
int gol_diag_absorbed(uint64_t* count, char* last, size_t cap);

#ifdef __cplusplus
}
#endif

#endif /* GOL_H */
