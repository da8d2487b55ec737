// rrte_hip.hip — C-ABI implementation (include/rrte_hip.h) of the MI355X-native
// replacement for rrte-renderer's Raytracer::render
// (Melthizar/RRTE crates/rrte-renderer/src/raytracer.rs:45-148).
//
// Host side: validate + lower rrte_scene_ir to device records (precomputing the
// per-object Transform matrices the reference rebuilds per ray,
// primitives.rs:303,421,522,628), cache them in HBM until the scene changes,
// launch the ray kernel, and (multi-GPU) gather interleaved row bands to the
// root over RCCL/xGMI.  No exception crosses the ABI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <future>
#include <limits>
#include <thread>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <new>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "bvh.hpp"
#include "jit.hpp"
#include "sdf_guard.hpp"
#include "ray_kernels.hpp"

using namespace rrte;

// Everything one launch of the ray kernel needs, decided on the host from the scene and parameters.
// A multi-frame launch (batched gather) is one plan whose KParams carry up to kMaxLaunchFrames
// cameras: blockIdx.y picks the frame (KParams::hot: grid (tile columns, frames, hot rows + tile rows)).
struct LaunchPlan {
    KParams k;
    int mode;
    bool cull, single;
    uint32_t num_prims, num_lights, num_materials;
    uint32_t gx, gy;
    int prof = 0;  // tile-profile slot (rrte_ctx::tprof): 0 whole frames / rank shares, 1 + i chunk i of a blocking frame
};

// A tile order composed off the render thread (plan_tile_order): the profile's shape key and the
// slot list (every tile, slowest first).
struct TilePlanResult {
    std::string key;
    std::vector<uint32_t> slots;
};

// A device resource that launches read asynchronously (a scene version, a tile-list version): the
// streams that launched work reading it since it became current, and -- once it is retired -- one
// event per such stream recorded at retirement, after that stream's last launch that read it.  The
// resource may be overwritten or freed once every event has completed.  No event is recorded per
// launch (an event after every launch put a gap between one stream's launches).
// Streams handed to the async entry points must therefore stay valid until the context has been
// synchronised (include/rrte_hip.h).
struct Retire {
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> events;
    size_t nev = 0;
    void use(hipStream_t st) {
        for (hipStream_t s : streams)
            if (s == st) return;
        streams.push_back(st);
    }
};

struct rrte_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    std::string err;
    // scene cache (device copy + the host bytes it was made from).  The device copy is versioned: a
    // ring of kSceneVersions buffer sets, so a scene change uploads into a version no frame in flight
    // reads (Retire) instead of draining the device; d_prims ... mesh_view alias the current version.
    std::vector<unsigned char> scene_key;
    // One scene version = ONE device allocation holding every array (objects, materials, lights, SDF
    // nodes, culling spheres, mesh BVH / triangles / normals / permutation at 256-B aligned offsets),
    // filled by ONE copy from a pinned staging buffer on the upload stream; a launch's stream waits
    // for that copy's event (once per stream and version), so a scene change never blocks the host
    // on the device.
    struct SceneBuf {
        uint8_t* d_buf = nullptr; size_t cap = 0;
        uint8_t* h_stage = nullptr; size_t cap_h = 0;  // pinned
        hipEvent_t ev_up = nullptr;                      // the version's upload copy done
        std::vector<hipStream_t> ordered;                // streams already made to wait for ev_up
        Retire ret;
    };
    static constexpr int kSceneVersions = 4;
    SceneBuf sb[kSceneVersions];
    int sb_cur = -1;
    hipStream_t upload_stream = nullptr;  // scene and tile-list H2D copies (never queued behind frames or gathers)
    DPrim* d_prims = nullptr;
    DMaterial* d_mats = nullptr;
    DLight* d_lights = nullptr;
    rrte_sdf_node* d_nodes = nullptr;
    float4* d_bounds = nullptr;
    MeshView mesh_view{};
    // device buffers replaced by larger ones while launches in flight may still read them: freed at
    // the next point where the context is idle (rrte_hip_synchronize, rrte_hip_destroy) instead of by a
    // hipFree that could wait on the device
    std::vector<void*> graveyard;
    void *h_warm = nullptr, *d_warm = nullptr;  // the upload stream's warm-up copy (rrte_hip_create)
    Retire launched;                 // every stream that launched a frame since the last synchronisation
    uint32_t n_prims = 0, n_mats = 0, n_lights = 0, n_nodes = 0;
    // frame buffers for the blocking entry points
    uint32_t* d_rgba = nullptr; size_t cap_rgba = 0;
    float4* d_f32 = nullptr; size_t cap_f32 = 0;
    unsigned long long* d_counters = nullptr;   // shadow rays, kCounterShards x kCounterStride (accumulating)
    unsigned long long* h_counters = nullptr;   // pinned copy
    unsigned long long shadow_base = 0;         // value at the start of the last frame
    // The blocking frame returns once the frame itself is complete; its counter copy lands after that
    // and is folded into rrte_stats when they are read (rrte_hip_stats) -- two pinned copy slots, so a
    // frame's copy never overwrites the one of the frame before it while that is unread
    unsigned long long* h_counters2 = nullptr;
    hipEvent_t ev_ctr[2] = {};        // slot's copy landed
    hipEvent_t ev_done = nullptr;     // the blocking frame complete (before its counter copy)
    bool ctr_pending = false;         // the last frame's counts are in slot ctr_slot, not yet in stats
    int ctr_slot = 0;
    // streams that have waited for the pending counter copy (issue_launch): a frame launched on another
    // stream than the context's must not add shadow rays to the counters while the blocking frame's
    // snapshot of them is still being copied
    std::vector<hipStream_t> ctr_ordered;
    // multi-GPU
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    int comm_size = 0;               // ranks of the RCCL communicator (nranks may be emulated, RRTE_EMULATE_RANK)
    uint32_t* d_gather = nullptr; size_t cap_gather = 0;
    uint32_t* d_full = nullptr; size_t cap_full = 0;
    static constexpr int kSlabs = 16;  // per-frame gathers (batch 1) that may be in flight at once
    hipEvent_t ev_gath[kSlabs] = {};
    hipStream_t slab_stream[kSlabs] = {};  // stream of the slab's last user (nullptr: never used)
    uint32_t* d_slab[kSlabs] = {};
    size_t cap_slab[kSlabs] = {};
    // the last collective issued (either form): gathers must run in issue order on every rank
    hipStream_t last_gather_stream = nullptr;
    hipEvent_t last_gather_ev = nullptr;
    // Batched gather (rrte_hip_set_gather_batch, B > 1): a frame call only plans its render (camera,
    // tile rectangles); every B frames (or at rrte_hip_flush / synchronize / a scene or parameter
    // change) the batch renders in multi-frame launches (blockIdx.y = frame, up to kMaxLaunchFrames
    // per launch) on the slab's render stream into the send slab, and the comm stream gathers all B
    // frames to the root in ONE ncclGather and de-interleaves them.  Every collective is issued on
    // the one comm stream, in program order; slab k's render stream overlaps slab k-1's gather.
    static constexpr int kMaxBatch = 16, kBatchSlabs = 6;
    static_assert(kMaxBatch == sizeof(rrte::DeinterleaveTargets::full) / sizeof(uint32_t*), "batch targets");
    uint32_t gather_batch = 1;
    hipStream_t comm_stream = nullptr;
    hipStream_t render_stream[kBatchSlabs] = {};
    struct Batch {
        uint32_t n = 0, cap = 0;             // frames planned into it / frames it was opened for
        uint32_t rendered = 0;               // frames [0, rendered) already launched into the send slab
        bool in_place = false;               // root: its bands rendered straight into the frames (RGBA8)
        bool per_frame = false;              // each frame launched at its call (not at the batch's close)
        uint32_t width = 0, height = 0, band = 0;
        BandMap bm{};                        // the batch's band partition (a frame with another closes it)
        int root = 0;
        bool rgb24 = false;
        size_t slice = 0;                    // bytes of one frame of one rank (256-B aligned)
        LaunchPlan plan;                     // frame 0's plan; frame j's camera in cam[j % kMaxLaunchFrames]
        FrameCam cam[kMaxBatch];
        uint32_t* full[kMaxBatch] = {};      // root: each frame's caller buffer
        uint32_t nsrc = 0;                   // distinct caller streams of the batch's frames
        hipStream_t src[kMaxBatch] = {};
        hipEvent_t ev_src[kMaxBatch] = {};   // recorded on src[i] at the flush
    } batch;
    int bslot = 0;
    bool env_comm_priority = true;           // RRTE_COMM_PRIORITY=0: comm stream at default priority (A/B)
    int batch_slabs = 3;                     // slabs in the ring (RRTE_BATCH_SLABS, A/B: 1..kBatchSlabs; 3 measured
                                             // best against 4 and 6, tools/runs/r03_call16.sh)
    hipEvent_t ev_batch[kBatchSlabs] = {};   // the slab's last batch gathered and de-interleaved
    hipEvent_t ev_render[kBatchSlabs] = {};  // the slab's last batch rendered
    uint8_t* d_bsend[kBatchSlabs] = {};
    size_t cap_bsend[kBatchSlabs] = {};
    uint8_t* d_brecv[kBatchSlabs] = {};
    size_t cap_brecv[kBatchSlabs] = {};
    uint64_t gather_frames = 0;
    // Collective failure detection: every wait for a gather is bounded by comm_timeout_ms
    // and polls ncclCommGetAsyncError; a gather that fails or does not complete aborts the communicator
    // (ncclCommAbort) and every later gather call returns RRTE_RCCL_ERROR until rrte_hip_comm_init.
    uint32_t comm_timeout_ms = 30000;
    bool comm_failed = false;
    std::string comm_fail_msg;
    uint64_t gathers_issued = 0;       // collectives issued on this communicator (both forms)
    hipEvent_t ev_poll[3 + kBatchSlabs] = {};  // bounded waits: the context's streams + the last gather
    // RRTE_FAULT_STALL_GATHER=N (fault injection, tests only): the N-th collective on this context is
    // preceded on its stream by a kernel that spins until the host releases it (or 5 s pass) -- a
    // stalled peer as seen from this rank.
    uint64_t fault_stall_at = 0;
    uint32_t* h_stall = nullptr;       // pinned, device-visible release flag
    bool stall_armed = false;
    // Blocking drop-in path (rrte_hip_render into a host buffer, Raytracer::render's signature): render,
    // then one pageable hipMemcpy (the runtime's path runs at PCIe rate, ~53 GB/s, tools/micro/d2h.hip).
    // Measured and rejected: a band copy kernel beside the render, and touching the
    // caller's fresh pages from host threads while the render runs.
    rrte_stats stats{};
    bool pending_kernel_timing = false;
    uint64_t pending_primary = 0;
    // scene-specialised kernels (jit.hip)
    int jit_mode = RRTE_JIT_AUTO;
    // environment switches, read once at rrte_hip_create (diagnostics / A-B runs / tests)
    uint32_t env_debug = 0;       // RRTE_DEBUG ablation bits
    int env_cull = -1;            // RRTE_CULL: -1 unset, 0 off, 1 on
    bool env_tile_cull = true;    // RRTE_TILE_CULL=0: no camera-ray tile culling (A/B, tests)
    bool env_force_gather = false;  // RRTE_FORCE_GATHER=1
    bool env_gather_rgba = false;   // RRTE_GATHER_RGB24=0: gather slabs always RGBA8
    bool env_band_sky = true;       // RRTE_BAND_SKY=0: the plain band interleave (band_layout)
    bool env_gather_self = false;   // RRTE_GATHER_SELF=1 (tests): the root sends its own bands to itself
                                    // through RCCL and expands them like a peer's (the 1-GPU check of the
                                    // send / recv / expand path)
    uint32_t env_guard_leaves = 2;  // RRTE_CSG_GUARDS: 0 = off, N = smallest guarded operand (leaves)
    bool env_wg256 = false;           // RRTE_WG64=0: specialised kernels in 256-thread workgroups (A/B only)
    int emu_nranks = 0, emu_rank = 0;  // RRTE_EMULATE_RANK=N:R: render_async renders rank R's bands of N (diagnostic)
    // RRTE_EMULATE_PEERS=N (tests, one GPU): a 1-rank communicator acts as the root of N ranks, and the
    // root renders every peer's packed share (exactly what RRTE_EMULATE_RANK=N:q renders, RGB24 slab
    // included) into peer q's receive slot where ncclRecv would have put it; the real expansion
    // (deinterleave_batch_kernel, skip_rank = root) then composes the frames -- the q >= 1 side of the
    // multi-GPU product path without the link
    int emu_peers = 0;
    uint64_t scene_gen = 0;       // bumped whenever the cached scene changes
    uint32_t scene_feat = kFeatAll;  // the cached scene's features (kFeat*): its generic kernel variant
    bool env_generic_all = false;    // RRTE_GENERIC_ALL=1: the all-features generic kernel for every scene (A/B, tests)
    // Batched gathers render the batch's frames in multi-frame launches at its close (default), or with
    // RRTE_BATCH_LAUNCH=0 each frame at its call (its own launch on the caller's stream: the root in
    // place, a peer into its slot of the send slab) with only the exchange batched -- measured slower
    // for rank shares (a launch of 1/N of a frame lasts as long as its slowest tile, so
    // per-frame launches are tail-bound; 8 frames per launch overlap their tails)
    bool env_batch_launch = true;
    // Blocking drop-in path into PINNED host memory (hipHostMalloc'd by the caller, or registered with
    // rrte_hip_host_register): the kernel stores the frame straight into the caller's buffer over PCIe
    // while it renders, instead of a render followed by one 8.3 MB D2H copy.  RRTE_BND_ZEROCOPY=0 turns
    // it off (A/B).  Pageable buffers keep the copy.
    bool env_bnd_zerocopy = true;
    uint32_t tile_shift = 3;          // tile shape of the launch being planned (KParams::tile_shift)
    bool env_zc_system_store = true;  // ... their pixel stores at system scope (RRTE_ZC_SYSTEM_STORE=0: plain, A/B)
    uint32_t zc_tile_shift = 5;       // ... of zero-copy blocking frames (RRTE_ZC_TILE_SHIFT: 3 / 4 / 5 / 6)
    struct HostReg { void* p; size_t bytes; };
    std::vector<HostReg> host_regs;   // rrte_hip_host_register'ed ranges (unregistered at destroy)
    struct { uint64_t gen; int mode, jit_mode; bool cull, single, topo, uniform, valid; JitKernel* k; } jit_last{};
    // Guard flavour of the scene-specialised kernel (device_scene.hpp RRTE_GUARD_UNIFORM): the correctly
    // rounded sequences' rare fallbacks as wave-uniform branches on a ballot (fewer scalar-unit
    // instructions, a longer dependent chain) or as divergent branches (measured, DESIGN.md §13: frame
    // streams -1.8 %, a lone frame +12 %).  RRTE_GUARD_POLICY: 0 divergent everywhere (default), 1
    // uniform everywhere, 2 uniform for the streaming entry points (async, gather) and divergent for
    // the blocking frame.
    bool jit_stream = true;         // the current call streams frames (false inside rrte_hip_render)
    int env_guard_policy = 0;
    uint64_t same_scene_renders = 0;             // consecutive renders of the cached scene
    // topology kernels (jit.hip JitTopo): the cached scene's topology key and structural decisions, and
    // how many consecutive scene changes kept that topology (value edits: an animation)
    int env_jit_topo = 2;                        // RRTE_JIT_TOPO: 0 full only, 1 topology only, 2 adaptive
    std::string topo_key;
    JitTopo topo;
    uint64_t value_edits = 0;
    std::vector<DPrim> h_prims;                  // host copy of the lowered scene (JIT source)
    std::vector<float4> h_bounds;                // host copy of the per-object culling spheres
    std::vector<DMaterial> h_mats;
    std::vector<DLight> h_lights;
    std::vector<rrte_sdf_node> h_nodes;
    std::unordered_map<std::string, JitKernel> jit_cache;  // failed compiles cached with fn == nullptr
    std::unordered_map<std::string, std::future<JitCode>> jit_pending;  // AUTO: background compiles
    std::string jit_log;
    // RRTE_HOST_PROFILE=1 (diagnostics): host time per section of rrte_hip_render_gather_async,
    // printed to stderr by rrte_hip_destroy
    bool host_prof = false;
    uint32_t env_diag_skip = 0;  // RRTE_DIAG_SKIP (1-rank timing diagnostics only): 1 no ncclGather, 2 no
                                 // de-interleave, 4 no comm-stream waits -- results are wrong
    double hp[16] = {};  // [0, 9): gather frames; [10, 15): asynchronous frames (rrte_hip_render_async)
    uint64_t hpa_frames = 0;
    double hpu[9] = {};     // scene uploads (upload_scene), RRTE_HOST_PROFILE sections (names at rrte_hip_destroy)
    uint64_t hpu_n = 0;
    bool hpa_cur = false;  // inside rrte_hip_render_async (its sections go to hp[10..15))
    uint64_t hp_frames = 0;
    // RRTE_TRACE=1 (diagnostics): every event record / stream wait / launch of the frame paths with its
    // stream and event, host-timestamped, printed to stderr by rrte_hip_destroy (matched against a
    // rocprofv3 kernel trace by launch order)
    bool trace = false;
    struct TraceRec { double us; const char* what; const void* st; const void* ev; uint32_t a, b; };
    std::vector<TraceRec> trace_log;
    std::chrono::steady_clock::time_point trace_t0 = std::chrono::steady_clock::now();
    // Tile order (KParams::hot).  Every kTileReprofile-th launch of one launch shape (size, rows, band
    // mapping, mode, kernel) times each tile of its frame 0 on the device and copies the durations back
    // asynchronously; once they have arrived, later launches of that shape dispatch every tile slowest
    // first (longest-processing-time order; RRTE_TILE_ORDER=1: only the 1024 slowest first, then image
    // order).  The order never changes a pixel, only when each tile starts.  RRTE_TILE_ORDER=0 turns it
    // off (A/B, tests).
    struct TileProfile {
        std::string key;                 // launch shape the tile list belongs to
        std::string pending_key;         // shape of the profile in flight
        bool pending = false;
        hipEvent_t ev = nullptr;         // the profile's D2H copy done
        uint32_t* d_cost = nullptr; size_t cap_d = 0;
        uint32_t* h_cost = nullptr; size_t cap_h = 0;  // pinned
        uint32_t tiles = 0, tiles_x = 0;                 // of the pending profile
        bool fixed = false;              // RRTE_TILE_ORDER=2 list
        std::vector<uint32_t> slots;     // packed hot_pack slots in dispatch order (every tile once)
        // device copies of slot lists (KParams::hot): a pool of immutable versions, one per upload.  The
        // current version is retired (Retire) when the next one is uploaded; an upload takes a retired
        // version whose launches have all completed, and when none has, the launch keeps the current
        // list (a stale order renders the same pixels) -- no render call ever waits for one.
        static constexpr int kVersions = 16;
        uint32_t* d_list[kVersions] = {};
        size_t cap_list[kVersions] = {};  // words
        Retire ret[kVersions];
        hipEvent_t ev_up[kVersions] = {};                 // the version's upload copy done
        std::vector<hipStream_t> ordered[kVersions];     // streams already made to wait for ev_up
        // pinned staging, one slice of `arena_words` per version in ONE page-locked allocation (one
        // hipHostMalloc per growth, not one per version): a version's slice is rewritten only when the
        // version is reused, i.e. after every launch that read it -- each of which waited for its copy
        // (ev_up); the arena grows only when no copy out of it is pending
        uint32_t* h_arena = nullptr;
        size_t arena_words = 0;
        int cur = -1;                    // version holding `slots` (-1: not uploaded)
        uint64_t launches = 0;           // launches of `key` since its last profile
        uint64_t profiles = 0;           // completed profiles
        uint64_t uploads = 0;            // list versions uploaded
        uint64_t cam_sig = 0;            // camera of the last profiled launch (frame 0's FrameCam)
        std::future<TilePlanResult> work;  // composition of the last profile's order (worker thread)
        bool working = false;
    };
    // One tile-order state per launch shape that alternates within a frame: slot 0 for whole frames
    // and rank shares, slot 1 + i for row chunk i of a blocking frame (render_chunked)
    // tile-profile slots: 0 frames into device buffers and the copy path, 1..kBndChunksMax the row
    // chunks of render_chunked, kZcProf zero-copy frames (their 32x2 tiles are another launch shape:
    // an engine alternating copy-path and zero-copy frames must not re-profile every frame)
    static constexpr int kBndChunksMax = 8, kZcProf = 1 + kBndChunksMax, kProfSlots = 2 + kBndChunksMax;
    TileProfile tprof[kProfSlots];
    // Blocking drop-in path (rrte_hip_render into a host buffer): the frame renders as row chunks on
    // streams of their own, and each chunk's D2H starts as soon as that chunk is done (render_chunked)
    // RRTE_BND_CHUNKS (default 1: one launch, then one copy).  Measured slower so far:
    // every chunk holding object rows is bound by its own slowest tile (~100 us), and the chunks'
    // launches start 7-17 us apart, so the copies cannot start before ~140 us
    int bnd_chunks = 1;
    hipStream_t bnd_stream[kBndChunksMax] = {};
    hipStream_t bnd_copy = nullptr;
    hipEvent_t ev_bchunk[kBndChunksMax] = {};
    hipEvent_t ev_bcopy = nullptr;
    bool env_tile_order = true;
    bool env_tile_order_fixed = false;  // RRTE_TILE_ORDER=2: a fixed scrambled permutation of the tiles (tests)
    // RRTE_NOCOMM_WAIT_MS: limit of device waits without a communicator (0 = none).  Nothing can stall
    // a frame without one, so the default is far above any frame (10 minutes): a hung or faulted kernel
    // still ends rrte_hip_synchronize / host_unregister / destroy with RRTE_HIP_ERROR
    uint32_t env_nocomm_wait_ms = 600000;
    // Retire sets / re-profile intervals shortened for tests (RRTE_TEST_RECYCLE=1: a tile-list version
    // per launch, so the version pool wraps within a few frames)
    bool env_test_recycle = false;
    int env_fault_bad_slot = 0;  // RRTE_FAULT_BAD_SLOT: 1 a tile-list slot, 2 an object kind (with RRTE_DEBUG bit 2)
    std::string dump_path;  // RRTE_DUMP_SCENE: every render call's scene + params into this file (scene_io.hip)
    // band partition of the last multi-GPU frame (frame_band_map)
    struct {
        bool valid = false;
        uint64_t gen = 0;
        uint32_t w = 0, h = 0, band = 0;
        int nranks = 0, root = 0, rank = 0;
        rrte_camera cam{};
        BandMap m{};
        uint32_t rows = 0, cap = 0;  // this rank's rows; the most rows any rank owns (slab rows)
    } band_cache;
    // camera-ray tile rectangles of the last camera (fill_tile_rects)
    struct {
        bool valid = false;
        uint64_t gen = 0;
        uint32_t width = 0, height = 0, band = 0;
        rrte_camera cam{};
        uint32_t tile_cull = 0, tile_n = 0;
        uint32_t rect[32] = {};
    } tile_rect_cache;
};

static rrte_status flush_batch(rrte_ctx* c);
static rrte_status render_batch(rrte_ctx* c, bool at_flush);
static rrte_status wait_bounded(rrte_ctx* c);
static rrte_status poll_events(rrte_ctx* c, const hipEvent_t* ev, size_t n);
static rrte_status nccl_settle(rrte_ctx* c, ncclResult_t r, const char* what);

namespace {

// Host-section timer for RRTE_HOST_PROFILE (no clock reads when it is off).
struct HostSection {
    rrte_ctx* c;
    std::chrono::steady_clock::time_point t;
    explicit HostSection(rrte_ctx* ctx) : c(ctx) {
        if (c->host_prof) t = std::chrono::steady_clock::now();
    }
    void lap(int k) {
        if (!c->host_prof) return;
        const auto n = std::chrono::steady_clock::now();
        c->hp[k] += std::chrono::duration<double, std::micro>(n - t).count();
        t = n;
    }
};

constexpr size_t kCounterBytes = sizeof(unsigned long long) * kCounterShards * kCounterStride;

rrte_status fail(rrte_ctx* c, rrte_status st, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return st;
}

#define HIPCHK(ctx, expr)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail((ctx), RRTE_HIP_ERROR, "%s failed: %s", #expr, hipGetErrorString(e_));     \
    } while (0)

// (the communicator is non-blocking: ncclInProgress is settled by polling, nccl_settle)
#define NCCLCHK(ctx, expr)                                                                         \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess) {                                                                   \
            rrte_status s_ = nccl_settle((ctx), r_, #expr);                                        \
            if (s_ != RRTE_OK) return s_;                                                          \
        }                                                                                          \
    } while (0)

void trace_rec(rrte_ctx* c, const char* what, const void* st, const void* ev, uint32_t a = 0, uint32_t b = 0) {
    if (!c->trace) return;
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c->trace_t0).count();
    c->trace_log.push_back({us, what, st, ev, a, b});
}
hipError_t ev_record(rrte_ctx* c, hipEvent_t ev, hipStream_t st, const char* tag) {
    trace_rec(c, tag, st, ev);
    return hipEventRecord(ev, st);
}
hipError_t ev_wait(rrte_ctx* c, hipStream_t st, hipEvent_t ev, const char* tag) {
    trace_rec(c, tag, st, ev);
    return hipStreamWaitEvent(st, ev, 0);
}

// Device buffer of at least n elements; a smaller one goes to the graveyard (launches in flight may
// still read it; freed when the context is next idle).
template <typename T>
rrte_status ensure(rrte_ctx* c, T*& ptr, size_t& cap, size_t n) {
    if (n <= cap && ptr) return RRTE_OK;
    if (ptr) c->graveyard.push_back(ptr);
    ptr = nullptr;
    cap = 0;
    size_t want = n < 1 ? 1 : n;
    HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&ptr), want * sizeof(T)));
    cap = want;
    return RRTE_OK;
}

// Retire a resource (struct Retire): an event on every stream that read it since it became current.
// Events of an earlier retirement that have not completed yet are kept.
rrte_status retire(rrte_ctx* c, Retire& r) {
    size_t keep = 0;
    for (size_t i = 0; i < r.nev; ++i)
        if (hipEventQuery(r.events[i]) != hipSuccess) std::swap(r.events[keep++], r.events[i]);
    r.nev = keep;
    for (hipStream_t s : r.streams) {
        if (r.events.size() <= r.nev) {
            hipEvent_t e = nullptr;
            HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            r.events.push_back(e);
        }
        HIPCHK(c, hipEventRecord(r.events[r.nev], s));
        ++r.nev;
    }
    r.streams.clear();
    return RRTE_OK;
}

// True when every launch that read a retired resource has completed (no wait).
bool retired_done(const Retire& r) {
    for (size_t i = 0; i < r.nev; ++i)
        if (hipEventQuery(r.events[i]) != hipSuccess) return false;
    return true;
}

// Bounded wait for a retired resource (poll_events: RRTE_RCCL_ERROR if a gather it sits behind stalls).
rrte_status wait_retired(rrte_ctx* c, Retire& r) {
    if (retired_done(r)) {
        r.nev = 0;
        return RRTE_OK;
    }
    rrte_status st = poll_events(c, r.events.data(), r.nev);
    if (st == RRTE_OK) r.nev = 0;
    return st;
}

void destroy_events(Retire& r) {
    for (hipEvent_t e : r.events)
        if (e) (void)hipEventDestroy(e);
    r.events.clear();
    r.nev = 0;
    r.streams.clear();
}

// ---- glam restatement on the host (same algorithms as oracle/, see there) ----
void mat4_srt(const float trs[10], float m[16]) {
    float x = trs[3], y = trs[4], z = trs[5], w = trs[6];
    float x2 = x + x, y2 = y + y, z2 = z + z;
    float xx = x * x2, xy = x * y2, xz = x * z2;
    float yy = y * y2, yz = y * z2, zz = z * z2;
    float wx = w * x2, wy = w * y2, wz = w * z2;
    float sx = trs[7], sy = trs[8], sz = trs[9];
    const float cols[3][3] = {{1.0f - (yy + zz), xy + wz, xz - wy},
                              {xy - wz, 1.0f - (xx + zz), yz + wx},
                              {xz + wy, yz - wx, 1.0f - (xx + yy)}};
    const float sc[3] = {sx, sy, sz};
    for (int c = 0; c < 3; ++c) {
        for (int r = 0; r < 3; ++r) m[c * 4 + r] = cols[c][r] * sc[c];
        m[c * 4 + 3] = 0.0f * sc[c];
    }
    m[12] = trs[0]; m[13] = trs[1]; m[14] = trs[2]; m[15] = 1.0f;
}

// glam Mat4::inverse (glm cofactor form), transform.rs:55-57
void mat4_inverse(const float* a, float* out) {
    auto M = [a](int c, int r) { return a[c * 4 + r]; };
    const float coef[18] = {
        M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3), M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3),
        M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3), M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3),
        M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3), M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3),
        M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2), M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2),
        M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2), M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3),
        M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3), M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3),
        M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2), M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2),
        M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2), M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1),
        M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1), M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1)};
    // Fac_k = (c_a, c_a, c_b, c_c) in glm's numbering
    const float fac[6][4] = {{coef[0], coef[0], coef[1], coef[2]},     {coef[3], coef[3], coef[4], coef[5]},
                             {coef[6], coef[6], coef[7], coef[8]},     {coef[9], coef[9], coef[10], coef[11]},
                             {coef[12], coef[12], coef[13], coef[14]}, {coef[15], coef[15], coef[16], coef[17]}};
    const float vec[4][4] = {{M(1, 0), M(0, 0), M(0, 0), M(0, 0)},
                             {M(1, 1), M(0, 1), M(0, 1), M(0, 1)},
                             {M(1, 2), M(0, 2), M(0, 2), M(0, 2)},
                             {M(1, 3), M(0, 3), M(0, 3), M(0, 3)}};
    float inv[16];
    for (int i = 0; i < 4; ++i) {
        float sa = (i & 1) ? -1.0f : 1.0f, sb = -sa;
        inv[0 * 4 + i] = ((vec[1][i] * fac[0][i] - vec[2][i] * fac[1][i]) + vec[3][i] * fac[2][i]) * sa;
        inv[1 * 4 + i] = ((vec[0][i] * fac[0][i] - vec[2][i] * fac[3][i]) + vec[3][i] * fac[4][i]) * sb;
        inv[2 * 4 + i] = ((vec[0][i] * fac[1][i] - vec[1][i] * fac[3][i]) + vec[3][i] * fac[5][i]) * sa;
        inv[3 * 4 + i] = ((vec[0][i] * fac[2][i] - vec[1][i] * fac[4][i]) + vec[2][i] * fac[5][i]) * sb;
    }
    float d0 = M(0, 0) * inv[0], d1 = M(0, 1) * inv[4], d2 = M(0, 2) * inv[8], d3 = M(0, 3) * inv[12];
    float det = (d0 + d1) + (d2 + d3);
    float rdet = 1.0f / det;
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * rdet;
}

void to_affine12(const float* m16, float* m12) {
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 3; ++r) m12[c * 3 + r] = m16[c * 4 + r];
}

bool sdf_program_ok(const rrte_sdf_node* nodes, uint32_t count) {
    int sp = 0, pp = 0;
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t op = nodes[i].op;
        if (op >= RRTE_SDF_SPHERE && op <= RRTE_SDF_ELLIPSOID) {
            if (++sp > RRTE_SDF_MAX_STACK) return false;
        } else if (op >= RRTE_SDF_UNION && op <= RRTE_SDF_SMOOTH_INTERSECTION) {
            if (sp < 2) return false;
            --sp;
        } else if (op >= RRTE_SDF_BEND && op <= RRTE_SDF_WAVE) {
            if (++pp > RRTE_SDF_MAX_POINT_STACK) return false;
            if ((op == RRTE_SDF_BEND || op == RRTE_SDF_TWIST || op == RRTE_SDF_TAPER || op == RRTE_SDF_WAVE) &&
                (nodes[i].i[0] > 2 || nodes[i].i[1] > 2))
                return false;
            if (op == RRTE_SDF_NOISE && nodes[i].i[0] > RRTE_SDF_MAX_OCTAVES) return false;
        } else if (op == RRTE_SDF_POP_POINT) {
            if (pp < 1) return false;
            --pp;
        } else {
            return false;
        }
    }
    return sp == 1 && pp == 0;
}

rrte_status validate(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p) {
    if (!s || !p) return fail(c, RRTE_INVALID_ARG, "null scene or params");
    if (p->width == 0 || p->height == 0) return fail(c, RRTE_INVALID_ARG, "zero-sized frame %ux%u", p->width, p->height);
    if ((uint64_t)p->width * p->height > (1ull << 30)) return fail(c, RRTE_INVALID_ARG, "frame too large");
    if (p->samples_per_pixel == 0) return fail(c, RRTE_INVALID_ARG, "samples_per_pixel must be >= 1");
    if (p->mode > RRTE_MODE_LAMBERT_SHADOW) return fail(c, RRTE_INVALID_ARG, "unknown mode %u", p->mode);
    if (p->jitter > RRTE_JITTER_RANDOM) return fail(c, RRTE_INVALID_ARG, "unknown jitter %u", p->jitter);
    // (the high bits are the library's own per-launch flags, kFlagSlabRgb24 / kFlagHostStore)
    if (p->flags & ~(uint32_t)(RRTE_FLAG_F32_LINEAR | RRTE_FLAG_GATHER_OVERLAP))
        return fail(c, RRTE_INVALID_ARG, "unknown flags 0x%x", p->flags);
    if ((s->num_prims && !s->prims) || (s->num_lights && !s->lights) || (s->num_materials && !s->materials) ||
        (s->num_sdf_nodes && !s->sdf_nodes))
        return fail(c, RRTE_INVALID_ARG, "null array with nonzero count");
    if (s->camera.projection > RRTE_ORTHOGRAPHIC) return fail(c, RRTE_INVALID_ARG, "unknown projection");
    if ((s->num_mesh_vertices && !s->mesh_vertices) || (s->num_mesh_indices && !s->mesh_indices))
        return fail(c, RRTE_INVALID_ARG, "null mesh array with nonzero count");
    if (s->num_mesh_indices % 3) return fail(c, RRTE_INVALID_ARG, "mesh index count not a multiple of 3");
    if (s->num_mesh_indices / 3 >= (1u << 24)) return fail(c, RRTE_INVALID_ARG, "more than 2^24 mesh triangles");
    for (uint32_t i = 0; i < s->num_prims; ++i) {
        const rrte_prim& pr = s->prims[i];
        if (pr.kind > RRTE_PRIM_MESH) return fail(c, RRTE_UNSUPPORTED_PRIM, "prim %u: unknown kind %u", i, pr.kind);
        if (pr.kind == RRTE_PRIM_MESH) {
            if ((uint64_t)pr.sdf_first + pr.sdf_count > s->num_mesh_indices / 3)
                return fail(c, RRTE_INVALID_ARG, "prim %u: mesh triangle range out of bounds", i);
        }
        if (pr.kind == RRTE_PRIM_SDF) {
            if ((uint64_t)pr.sdf_first + pr.sdf_count > s->num_sdf_nodes)
                return fail(c, RRTE_INVALID_ARG, "prim %u: SDF node range out of bounds", i);
            if (!sdf_program_ok(s->sdf_nodes + pr.sdf_first, pr.sdf_count))
                return fail(c, RRTE_INVALID_ARG, "prim %u: malformed SDF program", i);
        }
    }
    for (uint32_t i = 0; i < s->num_lights; ++i)
        if (s->lights[i].kind > RRTE_LIGHT_AMBIENT)
            return fail(c, RRTE_UNSUPPORTED_PRIM, "light %u: unknown kind %u", i, s->lights[i].kind);
    for (uint32_t i = 0; i < s->num_materials; ++i)
        if (s->materials[i].kind > RRTE_MAT_EMISSIVE)
            return fail(c, RRTE_UNSUPPORTED_PRIM, "material %u: unknown kind %u", i, s->materials[i].kind);
    return RRTE_OK;
}

// Conservative world-space bounding sphere of one object for wave culling
// (ray_kernels.hpp, primary_cull/shadow_cull): every point the object's
// intersector can report lies inside it.  Radius +inf = never culled (planes,
// non-finite data).  Computed in double and inflated, so f32 rounding in the
// intersectors stays inside.
float4 prim_bound(const rrte_prim& in, const DPrim& d) {
    const double inf = __builtin_huge_val();
    double c[3] = {in.p[0], in.p[1], in.p[2]}, r = inf;
    bool local = true;  // bound given in object space (transformed below)
    switch (in.kind) {
    case RRTE_PRIM_SPHERE: r = fabs((double)in.p[3]); local = false; break;
    case RRTE_PRIM_TRIANGLE: {
        for (int k = 0; k < 3; ++k) c[k] = ((double)in.p[k] + in.p[3 + k] + in.p[6 + k]) / 3.0;
        r = 0.0;
        for (int v = 0; v < 3; ++v) {
            double dx = in.p[3 * v] - c[0], dy = in.p[3 * v + 1] - c[1], dz = in.p[3 * v + 2] - c[2];
            r = fmax(r, sqrt(dx * dx + dy * dy + dz * dz));
        }
        local = false;
        break;
    }
    case RRTE_PRIM_CUBE: {
        double sx = in.p[4], sy = in.p[5], sz = in.p[6];
        r = 0.5 * sqrt(sx * sx + sy * sy + sz * sz);
        break;
    }
    case RRTE_PRIM_CYLINDER:
    case RRTE_PRIM_CONE: {
        double rad = in.p[3], hh = 0.5 * in.p[4];
        r = sqrt(rad * rad + hh * hh);
        break;
    }
    case RRTE_PRIM_CAPSULE: r = 0.5 * fabs((double)in.p[4]) + fabs((double)in.p[3]); break;
    case RRTE_PRIM_SDF: r = fabs((double)in.p[3]); local = false; break;  // the sphere tracer's own bound
    default: break;                                                       // plane: unbounded
    }
    if (local && r < inf) {  // p' = M p: centre through xf, radius by the largest column norm
        double w[3];
        for (int k = 0; k < 3; ++k)
            w[k] = (double)d.xf[0 + k] * c[0] + (double)d.xf[3 + k] * c[1] + (double)d.xf[6 + k] * c[2] + d.xf[9 + k];
        double sn = 0.0;
        for (int col = 0; col < 3; ++col) {
            double a = d.xf[col * 3], b = d.xf[col * 3 + 1], e = d.xf[col * 3 + 2];
            sn = fmax(sn, sqrt(a * a + b * b + e * e));
        }
        r *= sn * (1.0 + 1e-5);  // M = R*S (mat4_srt): orthogonal columns, so |M v| <= max column norm * |v|
        c[0] = w[0]; c[1] = w[1]; c[2] = w[2];
    }
    double mag = fmax(fabs(c[0]), fmax(fabs(c[1]), fabs(c[2])));
    r = r * 1.001 + 1e-3 + 1e-5 * mag;
    if (!(r < 3e38) || !std::isfinite(c[0]) || !std::isfinite(c[1]) || !std::isfinite(c[2]))
        return make_float4(0.0f, 0.0f, 0.0f, __builtin_huge_valf());
    return make_float4((float)c[0], (float)c[1], (float)c[2], nextafterf((float)r, __builtin_huge_valf()));
}

// Lower the ABI records to device records (matrices precomputed once per
// object instead of per ray as in primitives.rs:303,421,522,628).
void lower_scene(const rrte_scene_ir* s, std::vector<DPrim>& prims, std::vector<DMaterial>& mats,
                 std::vector<DLight>& lights, std::vector<float4>* bounds = nullptr) {
    prims.assign(s->num_prims, DPrim{});
    if (bounds) bounds->assign(s->num_prims, float4{});
    for (uint32_t i = 0; i < s->num_prims; ++i) {
        const rrte_prim& in = s->prims[i];
        DPrim& o = prims[i];
        memset(&o, 0, sizeof o);
        o.kind = in.kind;
        o.material = in.material;
        o.sdf_first = in.sdf_first;
        o.sdf_count = in.sdf_count;
        o.sdf_max_steps = in.sdf_max_steps;
        o.sdf_step_scale = in.sdf_step_scale;
        o.sdf_hit_eps = in.sdf_hit_eps;
        memcpy(o.p, in.p, sizeof o.p);
        float m[16], inv[16];
        mat4_srt(in.trs, m);
        mat4_inverse(m, inv);
        to_affine12(m, o.xf);
        to_affine12(inv, o.inv);
        if (bounds) (*bounds)[i] = prim_bound(in, o);
    }
    mats.assign(s->num_materials, DMaterial{});
    for (uint32_t i = 0; i < s->num_materials; ++i) {
        static_assert(sizeof(rrte_material) == sizeof(DMaterial), "material layout");
        memcpy(&mats[i], &s->materials[i], sizeof(DMaterial));
    }
    lights.assign(s->num_lights, DLight{});
    for (uint32_t i = 0; i < s->num_lights; ++i) {
        const rrte_light& in = s->lights[i];
        DLight& o = lights[i];
        memset(&o, 0, sizeof o);
        o.kind = in.kind;
        o.intensity = in.intensity;
        o.range = in.range;
        o.linear = in.linear;
        o.quadratic = in.quadratic;
        o.inner_angle = in.inner_angle;
        o.outer_angle = in.outer_angle;
        memcpy(o.position, in.position, sizeof o.position);
        memcpy(o.direction, in.direction, sizeof o.direction);
        memcpy(o.color, in.color, sizeof o.color);
        for (int k = 0; k < 4; ++k) o.cI[k] = in.color[k] * in.intensity;  // Color * f32 (light.rs:189)
    }
}

// Upload the scene if it differs from the cached copy (the analogue of
// caching on Scene::is_dirty, crates/rrte-scene/src/lib.rs:310-312).  The key
// is the IR's bytes; mesh arrays enter it through (addresses, counts,
// mesh_version), or by content when mesh_version is 0.
struct MeshKey {
    const void* v;
    const void* i;
    uint64_t nv, ni, version;
};

// The key parts of a scene IR (compared byte for byte against the cached scene's key).
struct SceneKeyParts {
    const void* parts[7];
    size_t lens[7];
    size_t total;
    MeshKey mk;
};
void scene_key_parts(const rrte_scene_ir* s, SceneKeyParts& kp) {
    kp.mk = MeshKey{s->mesh_vertices, s->mesh_indices, s->num_mesh_vertices, s->num_mesh_indices, s->mesh_version};
    const size_t bmv = s->mesh_version ? 0 : sizeof(rrte_mesh_vertex) * s->num_mesh_vertices;
    const size_t bmi = s->mesh_version ? 0 : sizeof(uint32_t) * s->num_mesh_indices;
    const void* parts[7] = {s->prims, s->materials, s->lights, s->sdf_nodes, &kp.mk, s->mesh_vertices, s->mesh_indices};
    const size_t lens[7] = {sizeof(rrte_prim) * s->num_prims, sizeof(rrte_material) * s->num_materials,
                            sizeof(rrte_light) * s->num_lights, sizeof(rrte_sdf_node) * s->num_sdf_nodes,
                            sizeof(MeshKey), bmv, bmi};
    kp.total = 0;
    for (int i = 0; i < 7; ++i) {
        kp.parts[i] = parts[i];
        kp.lens[i] = lens[i];
        kp.total += lens[i];
    }
}

// True if `s` is the scene cached on the device (no upload needed).
bool scene_same(const rrte_ctx* c, const rrte_scene_ir* s) {
    SceneKeyParts kp;
    scene_key_parts(s, kp);
    if (c->scene_key.size() != kp.total) return false;
    const unsigned char* k = c->scene_key.data();
    for (int i = 0; i < 7; ++i) {
        if (kp.lens[i] && memcmp(k, kp.parts[i], kp.lens[i])) return false;
        k += kp.lens[i];
    }
    return true;
}

// The scene's topology -- what a topology kernel compiles in (jit.hip, ray_kernels.hpp TopoPrim /
// TopoNode / TopoLight) -- as a key, with its structural decisions in `topo`: object kinds and SDF
// node ranges, node ops and integer arguments (CSG-guard links included), light kinds, per-object
// SDF convexity (value-dependent for cones) and per-light cullability.  Also stores each SDF
// program's leaf scale (sdf_leaf_scale, the secant exit's error bound) in its first node's spare
// slot f[11], where a topology kernel reads it; no other code reads f[11].
std::string topology_of(const std::vector<DPrim>& prims, const std::vector<DLight>& lights,
                        std::vector<rrte_sdf_node>& nodes, JitTopo& topo) {
    std::string key;
    auto put = [&](uint32_t v) { key.append(reinterpret_cast<const char*>(&v), sizeof v); };
    put((uint32_t)prims.size());
    put((uint32_t)lights.size());
    put((uint32_t)nodes.size());
    topo.convex.assign(prims.size(), 0);
    topo.cullable.assign(lights.size(), 0);
    for (size_t i = 0; i < prims.size(); ++i) {
        const DPrim& p = prims[i];
        put(p.kind);
        put(p.sdf_first);
        put(p.sdf_count);
        if (p.kind == RRTE_PRIM_SDF && p.sdf_count && (size_t)p.sdf_first + p.sdf_count <= nodes.size()) {
            topo.convex[i] = sdf_convex(&nodes[p.sdf_first], p.sdf_count) ? 1 : 0;
            nodes[p.sdf_first].f[11] = sdf_leaf_scale(&nodes[p.sdf_first], p.sdf_count);
        }
        put(topo.convex[i]);
    }
    for (const rrte_sdf_node& n : nodes) {
        put(n.op);
        put(n.i[0]);
        put(n.i[1]);
        put(n.i[2]);
    }
    for (size_t i = 0; i < lights.size(); ++i) {
        topo.cullable[i] = light_record_cullable(lights[i]) ? 1 : 0;
        put(lights[i].kind);
        put(topo.cullable[i]);
    }
    return key;
}

// The features of a scene (kFeat*) that pick its generic kernel variant.
uint32_t scene_features(const std::vector<DPrim>& prims, const std::vector<rrte_sdf_node>& nodes) {
    uint32_t f = 0u;
    for (const DPrim& p : prims) {
        if (p.kind == RRTE_PRIM_MESH) f |= kFeatMesh;
        else if (p.kind == RRTE_PRIM_SDF) f |= kFeatSdf;
        else if (p.kind != RRTE_PRIM_SPHERE) f |= kFeatAnalytic;
    }
    for (const rrte_sdf_node& n : nodes)
        if (n.op >= 64u) f |= kFeatDeform;  // deformers and their point pops
    return f;
}

// RRTE_DEBUG bit 2 (diagnostics): the indices of the uploaded scene, checked on the DEVICE copy the
// kernels read (one thread per object, on the upload stream right after the copy): check-
// word bit 16 an object kind out of range, 32 an SDF node range outside the uploaded nodes, 64 a
// CSG-guard link outside its program (it must name a later node of the same program).  The host
// validated the caller's IR (validate); this catches a device copy that differs from it.
__global__ __launch_bounds__(64) void scene_records_check(const DPrim* prims, uint32_t np, const rrte_sdf_node* nodes,
                                                          uint32_t nn, unsigned long long* counters) {
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= np) return;
    const DPrim& pr = prims[i];
    uint32_t bad = 0u;
    if (pr.kind > RRTE_PRIM_MESH) {
        bad |= 16u;
    } else if (pr.kind == RRTE_PRIM_SDF) {
        if ((uint64_t)pr.sdf_first + pr.sdf_count > nn) {
            bad |= 32u;
        } else {
            for (uint32_t k = 0; k < pr.sdf_count; ++k) {
                const uint32_t link = nodes[pr.sdf_first + k].i[2];
                if (link != 0u && (link - 1u <= k || link - 1u >= pr.sdf_count)) {
                    bad |= 64u;
                    break;
                }
            }
        }
    }
    if (bad) atomicOr(counters + 1, (unsigned long long)bad);
}

rrte_status upload_scene(rrte_ctx* c, const rrte_scene_ir* s, hipStream_t st, double* upload_ms) {
    const size_t bn = sizeof(rrte_sdf_node) * s->num_sdf_nodes;
    SceneKeyParts kparts;
    scene_key_parts(s, kparts);
    const size_t key_len = kparts.total;
    const bool same = scene_same(c, s);
    if (!same && c->batch.rendered < c->batch.n) {
        // the open batch's frames render the cached scene: launch them before the scene changes.  Local
        // only (no gather): a rank's own preview render with another scene must not close a batch the
        // other ranks keep open
        rrte_status r = render_batch(c, false);
        if (r != RRTE_OK) return r;
    }
    *upload_ms = 0.0;
    if (same) {
        ++c->same_scene_renders;
        return RRTE_OK;
    }
    (void)st;  // the copy runs on the context's upload stream; launches wait for its event (issue_launch)
    const auto t_up0 = std::chrono::steady_clock::now();
    auto t_sec = t_up0;
    auto lap_up = [&](int i) {  // (RRTE_HOST_PROFILE)
        if (!c->host_prof) return;
        const auto n = std::chrono::steady_clock::now();
        c->hpu[i] += std::chrono::duration<double, std::micro>(n - t_sec).count();
        t_sec = n;
    };

    for (uint32_t k = 0; k < s->num_mesh_indices; ++k)
        if (s->mesh_indices[k] >= s->num_mesh_vertices)
            return fail(c, RRTE_INVALID_ARG, "mesh index %u out of range (%u vertices)", k, s->num_mesh_vertices);
    std::vector<DPrim> prims;
    std::vector<DMaterial> mats;
    std::vector<DLight> lights;
    std::vector<float4> bounds;
    lower_scene(s, prims, mats, lights, &bounds);
    lap_up(0);
    MeshData md;
    build_mesh_bvhs(s, prims.data(), md, bounds.data());
    if (md.too_deep) return fail(c, RRTE_UNSUPPORTED_PRIM, "mesh BVH deeper than the traversal stack");
    lap_up(1);
    // SDF programs with their exact CSG early-outs (sdf_guard.hpp); the key above stays the caller's IR
    std::vector<rrte_sdf_node> nodes = decorate_scene_sdf(s, c->env_guard_leaves);
    lap_up(2);
    JitTopo topo;
    std::string tkey = topology_of(prims, lights, nodes, topo);
    lap_up(3);

    // Frames in flight keep reading the current version: retire it and upload into the next version
    // of the ring once the frames that read THAT one have completed (normally long ago: a wait here
    // means more scene changes than versions within the frames in flight; bounded, like every wait
    // that may sit behind a gather)
    rrte_status r;
    if (c->sb_cur >= 0 && (r = retire(c, c->sb[c->sb_cur].ret)) != RRTE_OK) return r;
    const int nx = (c->sb_cur + 1) % rrte_ctx::kSceneVersions;
    rrte_ctx::SceneBuf& B = c->sb[nx];
    if ((r = wait_retired(c, B.ret)) != RRTE_OK) return r;
    c->same_scene_renders = 0;
    ++c->scene_gen;
    c->sb_cur = -1;  // (until the upload has completed: a failure below leaves no current version)
    c->scene_key.clear();
    // one allocation, one staging buffer, one copy (256-B aligned sub-arrays)
    struct Part { const void* src; size_t bytes; size_t off; };
    Part parts[9] = {{prims.data(), prims.size() * sizeof(DPrim), 0},
                     {mats.data(), mats.size() * sizeof(DMaterial), 0},
                     {lights.data(), lights.size() * sizeof(DLight), 0},
                     {nodes.data(), bn, 0},
                     {bounds.data(), bounds.size() * sizeof(float4), 0},
                     {md.nodes.data(), md.nodes.size() * sizeof(float4), 0},
                     {md.tris.data(), md.tris.size() * sizeof(float4), 0},
                     {md.norms.data(), md.norms.size() * sizeof(float4), 0},
                     {md.perm.data(), md.perm.size() * sizeof(uint32_t), 0}};
    lap_up(4);
    size_t total = 0;
    for (Part& pt : parts) {
        pt.off = total;
        total += (pt.bytes + 255u) & ~(size_t)255u;
    }
    total = std::max<size_t>(total, 256u);
    // the staging buffer may still feed this version's previous upload if no launch ever read it
    if (B.ev_up) HIPCHK(c, hipEventSynchronize(B.ev_up));  // (upload stream: copies only, bounded)
    if ((r = ensure(c, B.d_buf, B.cap, total)) != RRTE_OK) return r;
    if (B.cap_h < total) {
        if (B.h_stage) (void)hipHostFree(B.h_stage);  // (its copies have completed: ev_up above)
        B.h_stage = nullptr;
        B.cap_h = 0;
        HIPCHK(c, hipHostMalloc(reinterpret_cast<void**>(&B.h_stage), total, hipHostMallocDefault));
        B.cap_h = total;
    }
    if (!B.ev_up) HIPCHK(c, hipEventCreateWithFlags(&B.ev_up, hipEventDisableTiming));
    for (const Part& pt : parts)
        if (pt.bytes) memcpy(B.h_stage + pt.off, pt.src, pt.bytes);
    lap_up(5);
    hipStream_t us = c->upload_stream;  // (created with the context)
    // fault injection for the check below (RRTE_FAULT_BAD_SLOT=2 with RRTE_DEBUG bit 2): object 0's
    // kind out of range in the device copy only (kernels skip an unknown kind; the host copy stays valid)
    if (c->env_fault_bad_slot == 2 && (c->env_debug & 4u) && !prims.empty())
        reinterpret_cast<DPrim*>(B.h_stage + parts[0].off)->kind = 0xbadu;
    HIPCHK(c, hipMemcpyAsync(B.d_buf, B.h_stage, total, hipMemcpyHostToDevice, us));
    lap_up(6);
    if ((c->env_debug & 4u) && !prims.empty()) {
        hipLaunchKernelGGL(scene_records_check, dim3(((uint32_t)prims.size() + 63u) / 64u), dim3(64), 0, us,
                           reinterpret_cast<const DPrim*>(B.d_buf + parts[0].off), (uint32_t)prims.size(),
                           reinterpret_cast<const rrte_sdf_node*>(B.d_buf + parts[3].off), (uint32_t)nodes.size(),
                           c->d_counters);
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(B.ev_up, us));
    lap_up(7);
    B.ordered.clear();
    // host time to lower the scene and enqueue its upload (the copy itself is asynchronous)
    *upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_up0).count();
    uint8_t* d = B.d_buf;
    c->d_prims = reinterpret_cast<DPrim*>(d + parts[0].off);
    c->d_mats = reinterpret_cast<DMaterial*>(d + parts[1].off);
    c->d_lights = reinterpret_cast<DLight*>(d + parts[2].off);
    c->d_nodes = reinterpret_cast<rrte_sdf_node*>(d + parts[3].off);
    c->d_bounds = reinterpret_cast<float4*>(d + parts[4].off);
    c->mesh_view = MeshView{reinterpret_cast<float4*>(d + parts[5].off), reinterpret_cast<float4*>(d + parts[6].off),
                            reinterpret_cast<float4*>(d + parts[7].off), reinterpret_cast<uint32_t*>(d + parts[8].off)};
    c->sb_cur = nx;
    c->h_prims = prims;
    c->h_bounds = bounds;
    c->h_mats = mats;
    c->h_lights = lights;
    c->h_nodes = std::move(nodes);
    c->scene_feat = scene_features(c->h_prims, c->h_nodes);
    c->value_edits = (!c->topo_key.empty() && tkey == c->topo_key) ? c->value_edits + 1 : 0;
    c->topo_key = std::move(tkey);
    c->topo = std::move(topo);
    c->n_prims = s->num_prims;
    c->n_mats = s->num_materials;
    c->n_lights = s->num_lights;
    c->n_nodes = s->num_sdf_nodes;
    c->scene_key.resize(key_len);
    unsigned char* k = c->scene_key.data();
    for (int i = 0; i < 7; ++i) {
        if (kparts.lens[i]) memcpy(k, kparts.parts[i], kparts.lens[i]);
        k += kparts.lens[i];
    }
    lap_up(8);
    c->hpu_n += c->host_prof;
    return RRTE_OK;
}

KParams make_params(const rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, uint32_t rows) {
    KParams k;
    memset(&k, 0, sizeof k);
    k.width = p->width;
    k.height = p->height;
    k.spp = p->samples_per_pixel;
    k.max_depth = p->max_depth;
    k.jitter = p->jitter;
    k.seed = p->seed;
    k.flags = p->flags;
    k.num_prims = s->num_prims;
    k.num_lights = s->num_lights;
    k.num_materials = s->num_materials;
    k.rows = rows;
    k.band_rows = c->nranks > 1 ? p->band_rows : 0;
    k.nranks = (uint32_t)c->nranks;
    k.rank = (uint32_t)c->rank;
    k.sky_bands = 0;  // (the plain interleave; plan_launch applies a frame's BandMap)
    k.root_bands = 1;
    k.peer_bands = 1;
    memcpy(k.bg, p->background, sizeof k.bg);
    k.t_min = p->t_min;
    k.bias = p->shadow_bias;
    k.inv_gamma = 1.0f / p->gamma;                        // raytracer.rs:79 -> color.rs:60
    k.inv_spp = 1.0f / (float)p->samples_per_pixel;       // raytracer.rs:76
    k.nframes = 1;
    k.frame_stride = 0;
    const rrte_camera& cam = s->camera;
    FrameCam& fc = k.cam[0];
    fc.projection = cam.projection;
    memcpy(fc.cam_pos, cam.position, sizeof fc.cam_pos);
    memcpy(fc.cam_rot, cam.rotation, sizeof fc.cam_rot);
    fc.half_h = tanf(cam.fov * 0.5f);                     // camera.rs:104
    fc.aspect = cam.aspect_ratio;
    fc.ortho_l = cam.left; fc.ortho_r = cam.right; fc.ortho_b = cam.bottom; fc.ortho_t = cam.top;
    float trs[10] = {cam.position[0], cam.position[1], cam.position[2], cam.rotation[0], cam.rotation[1],
                     cam.rotation[2], cam.rotation[3], cam.scale[0], cam.scale[1], cam.scale[2]};
    float m[16];
    mat4_srt(trs, m);
    to_affine12(m, fc.cam_xf);
    k.debug = c->env_debug;  // RRTE_DEBUG ablation bits (profiling only)
    return k;
}

// Camera-ray tile culling (KParams::tile_rect, ray_kernels.hpp camera_tile_mask), perspective frames:
// for each of the first 32 objects, the 8x8-pixel tiles (16x16 for frames wider or taller than 2048)
// whose camera rays can reach its culling
// sphere (the conservative bound shadow culling uses: centre, radius).  In camera space a ray
// direction (x, y, -1) that meets the sphere projects, in the xz plane, onto a line through the eye
// that meets the sphere's disc there, so x lies between the tangents of that disc (likewise y in the
// yz plane).  Double precision, then 2 pixels of margin per side -- orders of magnitude above the f32
// error of the device's ray directions (~1e-6 of the field of view) and of random jitter's extent
// (inside the pixel).  A sphere that contains the eye or reaches the plane z = 0 keeps the whole
// frame.  Bit-identical results by construction: a skipped test is one every lane would miss
// (tests/test_gpu_parity.py test_camera_tile_culling_is_exact).
void fill_tile_rects_uncached(const rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, KParams& kk);

// The rectangles depend only on the camera, the frame size, the band height and the cached scene's
// bounds: frames of an unchanged camera reuse the last result (the double-precision trigonometry is
// most of a frame call's host time in the batched multi-GPU path).
void fill_tile_rects(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, KParams& kk) {
    auto& tc = c->tile_rect_cache;
    if (tc.valid && tc.gen == c->scene_gen && tc.width == p->width && tc.height == p->height &&
        tc.band == kk.band_rows && !memcmp(&tc.cam, &s->camera, sizeof tc.cam)) {
        kk.cam[0].tile_cull = tc.tile_cull;
        kk.cam[0].tile_n = tc.tile_n;
        memcpy(kk.cam[0].tile_rect, tc.rect, sizeof tc.rect);
        return;
    }
    fill_tile_rects_uncached(c, s, p, kk);
    tc.valid = true;
    tc.gen = c->scene_gen;
    tc.width = p->width;
    tc.height = p->height;
    tc.band = kk.band_rows;
    tc.cam = s->camera;
    tc.tile_cull = kk.cam[0].tile_cull;
    tc.tile_n = kk.cam[0].tile_n;
    memcpy(tc.rect, kk.cam[0].tile_rect, sizeof tc.rect);
}

void tile_rects(bool enabled, const std::vector<float4>& bounds, const rrte_scene_ir* s, const rrte_render_params* p,
                KParams& kk);
void fill_tile_rects_uncached(const rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, KParams& kk) {
    tile_rects(c->env_tile_cull, c->h_bounds, s, p, kk);
}
void tile_rects(bool enabled, const std::vector<float4>& bounds, const rrte_scene_ir* s, const rrte_render_params* p,
                KParams& kk) {
    FrameCam& k = kk.cam[0];
    const uint32_t band_rows = kk.band_rows;
    k.tile_cull = 0;
    // 8x8 tiles (one per wave) when their indices fit 8 bits and bands keep 8-row tiles whole,
    // else 16x16 blocks (four 8x8 workgroups)
    auto fits = [&](uint32_t sh) {
        const uint32_t t = 1u << sh;
        return (p->width + t - 1) / t <= 256 && (p->height + t - 1) / t <= 256 &&
               (band_rows == 0 || band_rows % t == 0);
    };
    const uint32_t sh = fits(3) ? 3u : (fits(4) ? 4u : 0u);
    if (!enabled || s->camera.projection != RRTE_PERSPECTIVE || sh == 0 || bounds.size() < s->num_prims)
        return;
    const uint32_t nbx = (p->width + (1u << sh) - 1) >> sh, nby = (p->height + (1u << sh) - 1) >> sh;
    const rrte_camera& cam = s->camera;
    double q[4] = {cam.rotation[0], cam.rotation[1], cam.rotation[2], cam.rotation[3]};
    const double qn = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (!(qn > 0.0) || !std::isfinite(qn)) return;
    for (double& v : q) v /= qn;
    const double hh = std::tan(0.5 * (double)cam.fov), hw = (double)cam.aspect_ratio * hh;
    if (!(hh > 0.0) || !(hw > 0.0) || !std::isfinite(hh) || !std::isfinite(hw)) return;
    // world -> camera: the inverse rotation (conjugate quaternion) of v - position
    auto to_cam = [&](const double v[3], double out[3]) {
        const double bx = -q[0], by = -q[1], bz = -q[2], w = q[3];
        const double vb = v[0] * bx + v[1] * by + v[2] * bz, k0 = w * w - (bx * bx + by * by + bz * bz);
        const double cx = by * v[2] - bz * v[1], cy = bz * v[0] - bx * v[2], cz = bx * v[1] - by * v[0];
        out[0] = v[0] * k0 + 2.0 * bx * vb + 2.0 * w * cx;
        out[1] = v[1] * k0 + 2.0 * by * vb + 2.0 * w * cy;
        out[2] = v[2] * k0 + 2.0 * bz * vb + 2.0 * w * cz;
    };
    const uint32_t n = s->num_prims < 32u ? s->num_prims : 32u;
    const double margin = 2.0;
    for (uint32_t i = 0; i < n; ++i) {
        const float4 b = bounds[i];
        uint32_t rect = 0u | ((nbx - 1) << 8) | (0u << 16) | ((nby - 1) << 24);  // whole frame
        const double R = (double)b.w;
        const double w[3] = {(double)b.x - cam.position[0], (double)b.y - cam.position[1], (double)b.z - cam.position[2]};
        double v[3];
        to_cam(w, v);
        const bool finite = std::isfinite(R) && std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]);
        if (finite && R >= 0.0 && v[2] < -R * 1.001 - 1e-6) {  // entirely in front of the eye (z < 0)
            // tangent slopes of the disc (centre (c, -d), radius R, d > R) seen from the origin:
            // tan(alpha -/+ beta) with tan alpha = c / d and tan beta = R / sqrt(D^2 - R^2), by the
            // angle-sum identity (no trigonometry: this runs per object for every new camera).  The
            // disc lies in z < 0, so both tangents point forward (|alpha +/- beta| < pi/2) and both
            // denominators are positive; a non-positive one (rounding at the limit) leaves that
            // side unbounded
            auto range = [&](double cc, double& lo, double& hi) {
                const double d = -v[2], h2 = cc * cc + d * d - R * R;
                const double inf = std::numeric_limits<double>::infinity();
                if (!(h2 > 0.0)) {
                    lo = -inf;
                    hi = inf;
                    return;
                }
                const double ta = cc / d, tb = R / std::sqrt(h2);
                const double dl = 1.0 + ta * tb, dh = 1.0 - ta * tb;
                lo = dl > 0.0 ? (ta - tb) / dl : -inf;
                hi = dh > 0.0 ? (ta + tb) / dh : inf;
            };
            double xl, xh, yl, yh;
            range(v[0], xl, xh);
            range(v[1], yl, yh);
            // ndc_x = x / hw, pixel x = (ndc_x + 1) W / 2 - 1/2;  ndc_y = y / hh, pixel y = (1 - ndc_y) H / 2 - 1/2
            const double W = p->width, H = p->height;
            const double px0 = (xl / hw + 1.0) * W * 0.5 - 0.5 - margin, px1 = (xh / hw + 1.0) * W * 0.5 - 0.5 + margin;
            const double py0 = (1.0 - yh / hh) * H * 0.5 - 0.5 - margin, py1 = (1.0 - yl / hh) * H * 0.5 - 0.5 + margin;
            if (std::isfinite(px0) && std::isfinite(px1) && std::isfinite(py0) && std::isfinite(py1)) {
                if (px1 < 0.0 || py1 < 0.0 || px0 > W - 1.0 || py0 > H - 1.0) {
                    rect = 0xFFu | (0xFFu << 16);  // bx0 = 255 > bx1 = 0: no block (block indices <= 255)
                } else {
                    auto blk = [sh](double px, uint32_t nb) {
                        const double b = std::floor(px / (double)(1u << sh));
                        return (uint32_t)std::min<double>(std::max<double>(b, 0.0), (double)(nb - 1));
                    };
                    rect = blk(px0, nbx) | (blk(px1, nbx) << 8) | (blk(py0, nby) << 16) | (blk(py1, nby) << 24);
                }
            }
        }
        k.tile_rect[i] = rect;
    }
    k.tile_n = n;
    k.tile_cull = sh;
}

constexpr uint32_t kMaxCycleBands = 8u;  // largest root_bands / peer_bands of a partition

uint32_t rows_for_rank(uint32_t height, uint32_t band_rows, int nranks, int rank, uint32_t sky = 0u,
                       uint32_t root_bands = 1u, uint32_t peer_bands = 1u) {
    if (nranks <= 1 || band_rows == 0) return height;
    const BandMap m{band_rows, (uint32_t)nranks, sky, root_bands, peer_bands};
    uint32_t nb = (height + band_rows - 1) / band_rows, rows = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        uint32_t lb = 0;
        if (band_owner(m, b, lb) != (uint32_t)rank) continue;
        uint32_t r0 = b * band_rows, r1 = r0 + band_rows < height ? r0 + band_rows : height;
        rows += r1 - r0;
    }
    return rows;
}

// The number of leading bands no object reaches (band_layout); 0 when it cannot be judged.
uint32_t sky_band_count(const rrte_camera& cam, const std::vector<float4>& bounds, uint32_t num_prims,
                        uint32_t height, uint32_t band_rows) {
    if (cam.projection != RRTE_PERSPECTIVE || bounds.size() < num_prims || num_prims == 0) return 0u;
    double q[4] = {cam.rotation[0], cam.rotation[1], cam.rotation[2], cam.rotation[3]};
    const double qn = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const double hh = std::tan(0.5 * (double)cam.fov), hw = (double)cam.aspect_ratio * hh;
    if (!(qn > 0.0) || !std::isfinite(qn) || !(hh > 0.0) || !(hw > 0.0) || !std::isfinite(hh * hw)) return 0u;
    for (double& v : q) v /= qn;
    auto to_cam = [&](const double v[3], double out[3]) {  // the inverse rotation (as fill_tile_rects)
        const double bx = -q[0], by = -q[1], bz = -q[2], w = q[3];
        const double vb = v[0] * bx + v[1] * by + v[2] * bz, k0 = w * w - (bx * bx + by * by + bz * bz);
        const double cx = by * v[2] - bz * v[1], cy = bz * v[0] - bx * v[2], cz = bx * v[1] - by * v[0];
        out[0] = v[0] * k0 + 2.0 * bx * vb + 2.0 * w * cx;
        out[1] = v[1] * k0 + 2.0 * by * vb + 2.0 * w * cy;
        out[2] = v[2] * k0 + 2.0 * bz * vb + 2.0 * w * cz;
    };
    double top = std::numeric_limits<double>::infinity();  // topmost image row any object reaches
    for (uint32_t i = 0; i < num_prims; ++i) {
        const float4 b = bounds[i];
        const double R = b.w;
        const double w[3] = {(double)b.x - cam.position[0], (double)b.y - cam.position[1], (double)b.z - cam.position[2]};
        double v[3];
        to_cam(w, v);
        const double D = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        if (!std::isfinite(R) || !std::isfinite(D) || D <= R * 1.0001) return 0u;  // unbounded / around the eye
        const double u[3] = {v[0] / D, v[1] / D, v[2] / D}, cos2 = 1.0 - (R / D) * (R / D);
        for (int col = 0; col <= 16; ++col) {
            // image-plane point (px, s, -1): inside the cone iff d = u.p > 0 and d^2 >= cos2 |p|^2
            const double px = (2.0 * col / 16.0 - 1.0) * hw, k = u[0] * px - u[2], mm = px * px + 1.0;
            const double A = u[1] * u[1] - cos2, B = 2.0 * u[1] * k, C = k * k - cos2 * mm;
            auto inside = [&](double s) { return u[1] * s + k > 0.0 && A * s * s + B * s + C >= -1e-12; };
            double cand[3] = {hh, -std::numeric_limits<double>::infinity(), -std::numeric_limits<double>::infinity()};
            const double disc = B * B - 4.0 * A * C;
            if (A != 0.0 && disc >= 0.0) {
                const double sq = std::sqrt(disc);
                cand[1] = (-B + sq) / (2.0 * A);
                cand[2] = (-B - sq) / (2.0 * A);
            } else if (A == 0.0 && B != 0.0) {
                cand[1] = -C / B;
            }
            std::sort(cand, cand + 3, [](double x, double y) { return x > y; });
            for (double sv : cand) {
                if (!(sv <= hh) || !(sv >= -hh) || !inside(sv)) continue;
                top = std::min(top, (1.0 - sv / hh) * height * 0.5 - 0.5);  // image row of ndc_y = s / hh
                break;
            }
        }
    }
    const double free_rows = top - band_rows;  // one band of margin
    const uint32_t nb = (height + band_rows - 1) / band_rows;
    uint32_t sky = free_rows > 0.0 ? (uint32_t)std::min<double>(std::floor(free_rows / band_rows), nb) : 0u;
    return sky >= nb ? 0u : sky;  // (nothing visible at all: the plain interleave)
}

// The band partition of a multi-GPU frame (BandMap, device_scene.hpp).  The leading "sky" bands --
// rows above every object's silhouette, where every camera ray misses (the cheapest rows of the
// frame) -- go to the root; the other bands go round robin, root_bands for the root per peer_bands
// for every peer, the pair chosen by a work model so the busiest rank is least busy.
// The silhouette top: per object, the cone of directions from the eye that meet its culling sphere,
// cut at 17 columns across the frame on the image plane (a quadratic per column, double precision),
// minus one band of margin.  This decides only WHICH rank renders a band -- never a pixel -- so the
// sampling need not be conservative.  Every rank computes the same partition from the same scene and
// camera (host arithmetic only).  RRTE_BAND_SKY=0: the plain interleave (sky 0, 1:1).
BandMap band_layout(const rrte_camera& cam, const std::vector<float4>& bounds, uint32_t num_prims, uint32_t width,
                    uint32_t height, uint32_t band_rows, int nranks, int root, bool enabled) {
    BandMap m{band_rows, (uint32_t)std::max(nranks, 1), 0u, 1u, 1u};
    if (!enabled || nranks <= 1 || root != 0 || band_rows == 0) return m;
    m.sky = sky_band_count(cam, bounds, num_prims, height, band_rows);
    // The root's round-robin share: the (root_bands, peer_bands) pair giving the smallest busiest rank
    // under a work model over the actual band counts, fitted to emulated rank frames of the 1080p
    // showcase: a non-sky row costs 1, a sky row kSkyCost (camera rays that miss), and the root spends
    // kExpandCost per peer row it receives and expands (RCCL receive + the RGB24 expansion); ties
    // keep the smaller cycle
    constexpr double kSkyCost = 0.15, kExpandCost = 0.09;
    const uint32_t nb = (height + band_rows - 1) / band_rows;
    // The choice depends on the sky count, not on the camera itself: a moving camera repeats a few sky
    // counts, so each (sky, frame height, band height, ranks) is searched once (the search over every
    // pair and band was most of a moving-camera frame call's host time)
    struct Choice { uint32_t sky, height, band_rows, nranks, a, b; };
    thread_local std::vector<Choice> memo;
    for (const Choice& ch : memo)
        if (ch.sky == m.sky && ch.height == height && ch.band_rows == band_rows && ch.nranks == (uint32_t)nranks) {
            m.root_bands = ch.a;
            m.peer_bands = ch.b;
            return m;
        }
    std::vector<double> load((size_t)nranks);
    double best = std::numeric_limits<double>::infinity();
    for (uint32_t a = 0; a <= kMaxCycleBands; ++a)
        for (uint32_t b = 1; b <= kMaxCycleBands; ++b) {
            if (a == 0 ? b != 1 : std::gcd(a, b) != 1) continue;  // (one representative per ratio)
            if (a == 0 && m.sky == 0) continue;                   // (the root would own nothing)
            const BandMap t{band_rows, (uint32_t)nranks, m.sky, a, b};
            std::fill(load.begin(), load.end(), 0.0);
            for (uint32_t band = 0; band < nb; ++band) {
                uint32_t lb = 0;
                const uint32_t rows = std::min(band_rows, height - band * band_rows), o = band_owner(t, band, lb);
                load[o] += band < m.sky ? kSkyCost * rows : (double)rows;
                if (o != 0) load[0] += kExpandCost * rows;
            }
            const double busiest = *std::max_element(load.begin(), load.end());
            if (busiest < best - 1e-9) best = busiest, m.root_bands = a, m.peer_bands = b;
        }
    if (memo.size() >= 64) memo.clear();
    memo.push_back(Choice{m.sky, height, band_rows, (uint32_t)nranks, m.root_bands, m.peer_bands});
    return m;
}


// Shadow-ray culling (ray_kernels.hpp, shadow_cull) for LAMBERT_SHADOW frames: one lane per object,
// so scenes of <= 64 objects; it pays where an occlusion test is expensive (sphere-traced SDF
// objects) and costs a few percent on all-analytic scenes (measured).  RRTE_CULL=0/1
// forces it off/on (A/B runs, tests).
// RRTE_CSG_GUARDS: unset = 2 (guard operands of >= 2 leaves), 0 = off, N = smallest guarded operand
uint32_t env_guard_setting() {
    const char* g = getenv("RRTE_CSG_GUARDS");
    return g ? (uint32_t)strtoul(g, nullptr, 0) : 2u;
}

int env_cull_setting() {
    const char* ce = getenv("RRTE_CULL");
    return ce ? (ce[0] != '0' ? 1 : 0) : -1;
}

bool cull_policy(const rrte_scene_ir* s, uint32_t mode, int env_cull) {
    if (mode != RRTE_MODE_LAMBERT_SHADOW || s->num_prims > 64) return false;
    if (env_cull >= 0) return env_cull != 0;
    for (uint32_t i = 0; i < s->num_prims; ++i)
        if (s->prims[i].kind == RRTE_PRIM_SDF) return true;
    return false;
}

// Scene-specialised kernel for the cached scene + mode, compiling it if the
// JIT policy says so; nullptr = use the generic kernel.
constexpr uint32_t kJitMaxPrims = 128, kJitMaxNodes = 1024;

// FULL or TOPOLOGY kernel (RRTE_JIT_TOPO, rrte_hip.h).  Adaptive: topology while the scene's values keep
// changing under one topology (one compile for a whole animation), full once the scene has been
// rendered unchanged for kJitFullAfter frames (until that full kernel is ready, the topology kernel).
constexpr uint64_t kJitFullAfter = 16;

bool jit_wants_topology(const rrte_ctx* c) {
    return c->env_jit_topo == 1 ||
           (c->env_jit_topo == 2 && c->value_edits >= 1 && c->same_scene_renders < kJitFullAfter);
}

std::string jit_key(const rrte_ctx* c, bool topo, int mode, bool cull, bool single, bool uniform) {
    std::string key(1, topo ? 'T' : 'F');
    if (topo) key += c->topo_key;
    else key.append(c->scene_key.begin(), c->scene_key.end());
    key.push_back((char)mode);
    key.push_back((char)cull);
    key.push_back((char)single);
    key.push_back((char)uniform);
    return key;
}

bool jit_uniform_guards(const rrte_ctx* c) { return c->env_guard_policy == 2 ? c->jit_stream : c->env_guard_policy == 1; }

// The cached kernel for `key`, compiling it if the JIT policy says so; nullptr = not available (yet).
JitKernel* jit_lookup(rrte_ctx* c, const std::string& key, bool topo, int mode, bool cull, bool single, bool uniform) {
    auto it = c->jit_cache.find(key);
    if (it != c->jit_cache.end()) return it->second.fn ? &it->second : nullptr;
    JitKernel jk;
    std::string log;
    auto pend = c->jit_pending.find(key);
    if (pend != c->jit_pending.end()) {
        // AUTO: a background compile of this kernel is running; keep the current kernel until it lands
        if (pend->second.wait_for(std::chrono::seconds(0)) != std::future_status::ready) return nullptr;
        const JitCode jc = pend->second.get();
        c->jit_pending.erase(pend);
        trace_rec(c, "jit: module load begin", nullptr, nullptr, (uint32_t)jc.code.size());
        const bool loaded = hipSetDevice(c->device) == hipSuccess && jit_load(jc, jk, log);
        trace_rec(c, "jit: module load end", nullptr, nullptr, loaded);
        if (!loaded) {
            c->jit_log = log;
            jk = JitKernel{};
        } else {
            c->stats.jit_compile_ms = jk.compile_ms;
        }
    } else {
        if (!(c->jit_mode == RRTE_JIT_ON || c->same_scene_renders >= 1 || topo)) return nullptr;
        if (c->jit_cache.size() >= 32) {
            // frames launched from these modules may still run on caller streams (a mode / cull /
            // sample-count change does not re-upload the scene, so upload_scene's sync has not run)
            // (bounded: RRTE_RCCL_ERROR surfaces at the next gather call if a stalled gather blocks it)
            if (hipSetDevice(c->device) != hipSuccess || retire(c, c->launched) != RRTE_OK ||
                wait_retired(c, c->launched) != RRTE_OK)
                return nullptr;
            for (auto& kv : c->jit_cache) jit_release(kv.second);
            c->jit_cache.clear();
            c->jit_last.valid = false;
        }
        std::string src = jit_source(c->h_prims.data(), (uint32_t)c->h_prims.size(), c->h_mats.data(),
                                     (uint32_t)c->h_mats.size(), c->h_lights.data(), (uint32_t)c->h_lights.size(),
                                     c->h_nodes.data(), (uint32_t)c->h_nodes.size(), mode, cull, single,
                                     topo ? &c->topo : nullptr);
        if (c->env_wg256) src = "#define RRTE_WG256 1\n" + src;
        if (uniform) src = "#define RRTE_GUARD_UNIFORM 1\n" + src;
        if (c->jit_mode == RRTE_JIT_AUTO) {
            // compile on a background thread (hiprtc only); frames keep running on the current kernel
            c->jit_pending.emplace(key, std::async(std::launch::async, [src]() { return jit_compile_code(src); }));
            return nullptr;
        }
        if (hipSetDevice(c->device) != hipSuccess || !jit_compile(src, jk, log)) {
            c->jit_log = log;  // stay on the generic kernel for this scene
            jk = JitKernel{};
        } else {
            c->stats.jit_compile_ms = jk.compile_ms;
        }
    }
    jk.topology = topo;
    auto& slot = c->jit_cache[key];
    slot = jk;
    return slot.fn ? &slot : nullptr;
}

JitKernel* jit_kernel_for(rrte_ctx* c, int mode, bool cull, bool single) {
    if (c->jit_mode == RRTE_JIT_OFF) return nullptr;
    auto& last = c->jit_last;  // per-frame fast path: same scene, mode, policy and kernel kind as the last frame
    const bool topo = jit_wants_topology(c);
    const bool uniform = jit_uniform_guards(c);
    if (last.valid && last.gen == c->scene_gen && last.mode == mode && last.cull == cull && last.single == single &&
        last.jit_mode == c->jit_mode && last.topo == topo && last.uniform == uniform)
        return last.k;
    if (c->h_prims.size() > kJitMaxPrims || c->h_nodes.size() > kJitMaxNodes) return nullptr;
    const std::string key = jit_key(c, topo, mode, cull, single, uniform);
    JitKernel* k = jit_lookup(c, key, topo, mode, cull, single, uniform);
    if (!k && !c->jit_cache.count(key)) {
        // not available yet (AUTO: not due, or compiling in the background): not remembered, asked again
        // next frame.  The full kernel of a scene that stopped changing: its topology kernel meanwhile
        if (!topo && c->env_jit_topo == 2 && c->value_edits >= 1) {
            auto it = c->jit_cache.find(jit_key(c, true, mode, cull, single, uniform));
            if (it != c->jit_cache.end() && it->second.fn) return &it->second;
        }
        return nullptr;
    }
    last.gen = c->scene_gen;
    last.mode = mode;
    last.jit_mode = c->jit_mode;
    last.cull = cull;
    last.single = single;
    last.topo = topo;
    last.uniform = uniform;
    last.k = k;
    last.valid = true;
    return k;
}

// Tile rows of a launch of `rows` rows (KParams::tile_shift: tiles 64 >> tile_shift rows high).
uint32_t tile_grid_rows(const KParams& k, uint32_t rows) {
    const uint32_t th = 64u >> k.tile_shift;
    return (rows + th - 1u) / th;
}

LaunchPlan plan_launch(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, uint32_t rows,
                       uint32_t internal_flags, uint32_t row0 = 0u, const BandMap* bm = nullptr) {
    LaunchPlan L;
    L.k = make_params(c, s, p, rows);
    if (bm && L.k.band_rows) {
        L.k.sky_bands = bm->sky;
        L.k.root_bands = bm->root_bands;
        L.k.peer_bands = bm->peer_bands;
    }
    L.k.row0 = row0;  // (image rows [row0, row0 + rows); band_rows == 0)
    L.k.flags |= internal_flags;
    L.mode = (int)p->mode;
    L.cull = cull_policy(s, p->mode, c->env_cull);
    // single-sample, single-bounce frames get the straight-line specialisation (SINGLE); others the
    // specialisation with runtime sample / bounce loops
    L.single = p->samples_per_pixel == 1 && (p->mode == RRTE_MODE_LAMBERT_SHADOW || p->max_depth <= 1);
    L.num_prims = s->num_prims;
    L.num_lights = s->num_lights;
    L.num_materials = s->num_materials;
    L.k.tile_shift = c->tile_shift;  // one tile per 64-thread workgroup (kBlockThreads): 8x8 unless overridden
    L.gx = (p->width + (1u << L.k.tile_shift) - 1u) >> L.k.tile_shift;
    L.gy = tile_grid_rows(L.k, rows);
    fill_tile_rects(c, s, p, L.k);
    return L;
}

// The band partition of one multi-GPU frame of this context (band_layout from the frame's camera-ray
// tile rectangles; `p` with its band_rows set).
// The band partition of a multi-GPU frame, this rank's rows under it and the slab rows (the most any
// rank owns); the last answer is kept (the same camera, scene, size, rank and rank count)
const BandMap& frame_band_map(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, int root,
                              uint32_t* rows = nullptr, uint32_t* cap = nullptr) {
    auto& bc = c->band_cache;
    if (!(bc.valid && bc.gen == c->scene_gen && bc.w == p->width && bc.h == p->height && bc.band == p->band_rows &&
          bc.nranks == c->nranks && bc.root == root && bc.rank == c->rank &&
          !memcmp(&bc.cam, &s->camera, sizeof bc.cam))) {
        bc.m = band_layout(s->camera, c->h_bounds, s->num_prims, p->width, p->height, p->band_rows, c->nranks, root,
                           c->env_band_sky);
        bc.valid = true;
        bc.gen = c->scene_gen;
        bc.w = p->width;
        bc.h = p->height;
        bc.band = p->band_rows;
        bc.nranks = c->nranks;
        bc.root = root;
        bc.rank = c->rank;
        bc.cam = s->camera;
        // every rank's rows in one pass over the bands (as rows_for_rank counts them)
        std::vector<uint32_t> per((size_t)c->nranks, 0u);
        if (c->nranks <= 1 || p->band_rows == 0) {
            per.assign((size_t)std::max(c->nranks, 1), p->height);
        } else {
            const uint32_t nb = (p->height + p->band_rows - 1) / p->band_rows;
            for (uint32_t b = 0; b < nb; ++b) {
                uint32_t lb = 0;
                const uint32_t r0 = b * p->band_rows, r1 = std::min(r0 + p->band_rows, p->height);
                per[band_owner(bc.m, b, lb)] += r1 - r0;
            }
        }
        bc.rows = per[(size_t)c->rank];
        bc.cap = *std::max_element(per.begin(), per.end());
    }
    if (rows) *rows = bc.rows;
    if (cap) *cap = bc.cap;
    return bc.m;
}

// Measured-cost tile order (rrte_ctx::TileProfile, KParams::hot).
constexpr uint64_t kTileReprofile = 256;  // launches of one shape between two profiles (each costs a list upload)
constexpr uint64_t kTileReprofileMoving = 32;  // ... when the camera has moved since the last profile

uint64_t fnv1a(const void* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ static_cast<const unsigned char*>(p)[i]) * 1099511628211ull;
    return h;
}

// Every tile of a profile (costs[0 .. n), tiles_x per row), slowest first (longest-processing-time
// order), as packed slots: a counting sort on 65536 cost buckets (ties in tile order), O(tiles) on the
// host.
std::vector<uint32_t> lpt_slots(const uint32_t* costs, uint32_t n, uint32_t tiles_x) {
    std::vector<uint32_t> slots;
    if (n == 0 || tiles_x == 0) return slots;
    uint32_t mx = 0;
    for (uint32_t i = 0; i < n; ++i) mx = std::max(mx, costs[i]);
    constexpr uint32_t B = 65536;
    std::vector<uint32_t> cnt(B + 1, 0u);
    auto bucket = [&](uint32_t c) { return B - 1 - (mx ? (uint32_t)((uint64_t)c * (B - 1) / mx) : 0u); };
    for (uint32_t i = 0; i < n; ++i) ++cnt[bucket(costs[i])];
    uint32_t acc = 0;
    for (uint32_t b = 0; b <= B; ++b) {
        const uint32_t c = cnt[b];
        cnt[b] = acc;
        acc += c;
    }
    slots.resize(n);
    for (uint32_t i = 0; i < n; ++i) slots[cnt[bucket(costs[i])]++] = hot_pack(i % tiles_x, i / tiles_x);
    return slots;
}

// RRTE_TILE_ORDER=2 (tests): every tile once in a fixed scrambled order -- slot k takes tile
// (k * stride) mod n for a stride near 0.618 n coprime with n -- so the list path runs on every launch
// without a profile.
std::vector<uint32_t> fixed_slots(uint32_t n, uint32_t tiles_x) {
    std::vector<uint32_t> slots(n);
    uint64_t stride = std::max<uint64_t>(1, (uint64_t)(0.618034 * n));
    auto gcd = [](uint64_t a, uint64_t b) { while (b) { const uint64_t t = a % b; a = b; b = t; } return a; };
    while (n > 1 && gcd(stride, n) != 1) ++stride;
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t i = (uint32_t)((k * stride) % n);
        slots[k] = hot_pack(i % tiles_x, i / tiles_x);
    }
    return slots;
}

// Words per XCD of a tile list of n slots stored XCD-major (KParams::hot_stride).
uint32_t hot_stride(uint32_t n) { return (n + 7u) / 8u; }

// Allocates what an upload of up to `words` list words needs -- the pinned staging arena and the device
// versions not yet allocated -- at profile time, so the first upload (inside a later render call)
// allocates nothing.  The copies run on the context's upload stream, created with the context: a
// stream's first use sets up its hardware queue (~8 ms measured, profiles/r06_engine_loop_trace.log),
// which must not land in a frame.  false = not now (a copy out of the arena is still pending).
bool reserve_hot_lists(rrte_ctx::TileProfile& tp, size_t words) {
    constexpr int K = rrte_ctx::TileProfile::kVersions;
    if (tp.arena_words < words) {
        for (int i = 0; i < K; ++i)
            if (tp.ev_up[i] && hipEventQuery(tp.ev_up[i]) != hipSuccess) return false;
        if (tp.h_arena) (void)hipHostFree(tp.h_arena);
        tp.h_arena = nullptr;
        tp.arena_words = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&tp.h_arena), K * words * sizeof(uint32_t), hipHostMallocDefault) !=
            hipSuccess)
            return false;
        tp.arena_words = words;
    }
    for (int i = 0; i < rrte_ctx::TileProfile::kVersions; ++i)
        if (!tp.d_list[i]) {
            if (hipMalloc(reinterpret_cast<void**>(&tp.d_list[i]), words * sizeof(uint32_t)) != hipSuccess) return false;
            tp.cap_list[i] = words;
        }
    return true;
}

// Uploads the composed slots into a free version of the device list; false leaves the launch on the
// current list (or in image order) -- it never waits for the device.  The current version is retired
// first; a version is free once every launch that read it has completed (struct Retire).  The copy
// runs on the list's own upload stream; its event orders every stream's first launch that reads the
// version after it (plan_tile_order), so every launch sees a whole list and no render call waits.
bool upload_hot_list(rrte_ctx* c, rrte_ctx::TileProfile& tp) {
    constexpr int K = rrte_ctx::TileProfile::kVersions;
    int pick = -1;
    for (int k = 1; k <= K && pick < 0; ++k) {  // the oldest retired version first
        const int v = (int)((tp.uploads + (uint64_t)k) % K);
        if (v != tp.cur && retired_done(tp.ret[v])) pick = v;
    }
    if (pick < 0) return false;
    trace_rec(c, "hot-list upload: begin", nullptr, nullptr, (uint32_t)pick);
    tp.ret[pick].nev = 0;
    const size_t n = tp.slots.size(), stride = hot_stride((uint32_t)n);
    const size_t words = 8u * stride;  // XCD-major (KParams::hot_stride)
    const size_t bytes = words * sizeof(uint32_t);
    if (tp.cap_list[pick] < words) {  // a larger frame: its launches have completed, the old buffer is idle
        if (tp.d_list[pick]) c->graveyard.push_back(tp.d_list[pick]);
        tp.d_list[pick] = nullptr;
        tp.cap_list[pick] = 0;
        if (hipMalloc(reinterpret_cast<void**>(&tp.d_list[pick]), bytes) != hipSuccess) return false;
        tp.cap_list[pick] = words;
    }
    trace_rec(c, "hot-list upload: device buffer", nullptr, nullptr, (uint32_t)pick);
    if (!reserve_hot_lists(tp, words)) return false;
    trace_rec(c, "hot-list upload: reserved", nullptr, nullptr, (uint32_t)pick);
    uint32_t* stage = tp.h_arena + (size_t)pick * tp.arena_words;
    for (size_t k = 0; k < n; ++k) stage[(k & 7u) * stride + (k >> 3)] = tp.slots[k];
    // fault injection for the device index check (tests): only where the check stops the wave first
    if (c->env_fault_bad_slot == 1 && (c->env_debug & 4u) && n) stage[0] = hot_pack(0u, 0xfff0u);
    if (!tp.ev_up[pick] && hipEventCreateWithFlags(&tp.ev_up[pick], hipEventDisableTiming) != hipSuccess) return false;
    trace_rec(c, "hot-list upload: staged", nullptr, nullptr, (uint32_t)pick);
    if (hipMemcpyAsync(tp.d_list[pick], stage, bytes, hipMemcpyHostToDevice, c->upload_stream) != hipSuccess)
        return false;
    trace_rec(c, "hot-list upload: copy queued", c->upload_stream, nullptr, (uint32_t)bytes);
    if (hipEventRecord(tp.ev_up[pick], c->upload_stream) != hipSuccess) return false;
    tp.ordered[pick].clear();
    if (tp.cur >= 0 && retire(c, tp.ret[tp.cur]) != RRTE_OK) return false;
    tp.cur = pick;
    ++tp.uploads;
    return true;
}

// Sets the plan's tile order (slot list, tile profile) for a launch of kernel `kern`; true when this
// launch is profiled (the caller copies the durations back after it).
bool plan_tile_order(rrte_ctx* c, LaunchPlan& L, const void* kern, hipStream_t st) {
    KParams& k = L.k;
    k.tiles_x = L.gx;
    k.hot = nullptr;
    k.hot_n = 0;
    k.hot_stride = 0;
    k.tile_cost = nullptr;
    // (RRTE_DEBUG bit 5 runs one workgroup in image-order numbering: no tile order; bit 4's per-wave
    // stamps work with it)
    if (!c->env_tile_order || c->env_wg256 || L.gx > 0xffffu || L.gy > 0xffffu || (k.debug & 32u)) return false;
    auto& tp = c->tprof[L.prof];
    std::string key(reinterpret_cast<const char*>(&kern), sizeof kern);
    const uint32_t shape[] = {k.width, k.height, k.rows, k.row0, k.band_rows, k.nranks, k.rank, k.spp, k.max_depth,
                              (uint32_t)L.mode, (uint32_t)L.cull, (uint32_t)L.single, k.tile_shift};
    key.append(reinterpret_cast<const char*>(shape), sizeof shape);
    const uint32_t tiles = L.gx * L.gy;
    if (tp.pending && hipEventQuery(tp.ev) == hipSuccess) {
        trace_rec(c, "tile plan: profile landed", st, nullptr);
        tp.pending = false;
        if (tp.pending_key == key) {
            // the order is composed on a worker thread from a copy of the durations: a whole frame's
            // counting sort takes ~0.5 ms of host time that a render call must not stall for
            std::vector<uint32_t> costs(tp.h_cost, tp.h_cost + tp.tiles);
            const uint32_t tx = tp.tiles_x;
            tp.work = std::async(std::launch::async, [key, costs = std::move(costs), tx]() {
                return TilePlanResult{key, lpt_slots(costs.data(), (uint32_t)costs.size(), tx)};
            });
            tp.working = true;
            tp.launches = 0;
            ++tp.profiles;
        }
    }
    if (tp.working && tp.work.wait_for(std::chrono::seconds(0)) == std::future_status::ready) {
        trace_rec(c, "tile plan: worker result", st, nullptr);
        TilePlanResult r = tp.work.get();
        tp.working = false;
        if (r.key == key && r.slots.size() == tiles) {  // (a result for another shape is dropped)
            tp.key = key;
            tp.slots = std::move(r.slots);
            tp.fixed = false;
            if (tp.cur >= 0 && retire(c, tp.ret[tp.cur]) != RRTE_OK) return false;
            tp.cur = -1;
        }
    }
    if (tp.key != key) {  // another shape: drop the list, profile as soon as the copy buffer is free
        tp.key = key;
        tp.slots.clear();
        tp.fixed = c->env_tile_order_fixed;
        if (tp.fixed) tp.slots = fixed_slots(tiles, L.gx);
        if (tp.cur >= 0 && retire(c, tp.ret[tp.cur]) != RRTE_OK) return false;
        tp.cur = -1;
        tp.launches = kTileReprofile;
    }
    if (tp.fixed) tp.launches = 0;  // RRTE_TILE_ORDER=2: the fixed list, never profiled
    // a moving camera moves the expensive tiles: re-profile after kTileReprofileMoving launches instead
    const uint64_t cam = fnv1a(&k.cam[0], offsetof(FrameCam, tile_cull));
    const bool moved = cam != tp.cam_sig;
    const uint64_t every = c->env_test_recycle ? 1 : kTileReprofile, moving = c->env_test_recycle ? 1 : kTileReprofileMoving;
    const bool profile = !tp.pending && (tp.launches >= every || (moved && tp.launches >= moving));
    ++tp.launches;
    // RRTE_TEST_RECYCLE=1: a new list version every launch (the fixed list re-uploaded), so the
    // version pool wraps within kVersions launches
    // (into a free version, retiring the current one; with none free the launch keeps the current list)
    if (c->env_test_recycle && tp.fixed && tp.cur >= 0) (void)upload_hot_list(c, tp);
    if (!tp.slots.empty() && tp.slots.size() == tiles && (tp.cur >= 0 || upload_hot_list(c, tp))) {
        auto& ord = tp.ordered[tp.cur];  // (first launch of this stream on the version: after its upload)
        if (tp.ev_up[tp.cur] && std::find(ord.begin(), ord.end(), st) == ord.end()) {
            if (ev_wait(c, st, tp.ev_up[tp.cur], "wait tile-list upload") != hipSuccess) return false;
            ord.push_back(st);
        }
        k.hot = tp.d_list[tp.cur];
        k.hot_n = (uint32_t)tp.slots.size();
        k.hot_stride = hot_stride(k.hot_n);
        tp.ret[tp.cur].use(st);
    }
    if (!profile) return false;
    if (ensure(c, tp.d_cost, tp.cap_d, tiles) != RRTE_OK) return false;
    if (tp.cap_h < tiles) {
        if (tp.h_cost) (void)hipHostFree(tp.h_cost);  // (no copy into it is pending: !tp.pending)
        tp.h_cost = nullptr;
        tp.cap_h = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&tp.h_cost), tiles * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess)
            return false;
        tp.cap_h = tiles;
    }
    if (!tp.ev && hipEventCreateWithFlags(&tp.ev, hipEventDisableTiming) != hipSuccess) return false;
    trace_rec(c, "tile profile: reserve lists", st, nullptr, tiles);
    if (!reserve_hot_lists(tp, 8u * (size_t)hot_stride(tiles))) return false;
    trace_rec(c, "tile profile: reserved", st, nullptr, tiles);
    k.tile_cost = tp.d_cost;  // every tile of frame 0 stores its duration (no clearing needed)
    tp.cam_sig = cam;
    tp.pending_key = key;
    tp.tiles = tiles;
    tp.tiles_x = L.gx;
    return true;
}

// Queues the profiled launch's copy-back on its stream (plan_tile_order returned true).
rrte_status finish_tile_order(rrte_ctx* c, const LaunchPlan& L, bool profile, hipStream_t st) {
    auto& tp = c->tprof[L.prof];
    if (!profile) return RRTE_OK;
    HIPCHK(c, hipMemcpyAsync(tp.h_cost, tp.d_cost, (size_t)tp.tiles * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(c, ev_record(c, tp.ev, st, "record tile-profile copy"));
    tp.pending = true;
    return RRTE_OK;
}

// The generic kernel variant for a scene with features `need` (kFeat*): the first of the
// precompiled feature sets F0, F1, F2 that covers it, else every feature (ray_kernels.hpp SceneView).
template <int MODE, bool CULL, uint32_t F0, uint32_t F1, uint32_t F2>
void launch_generic(uint32_t need, dim3 grid, dim3 block, hipStream_t st, const KParams& k, const SceneView& sv,
                    const Cull& cl, uint32_t* d_rgba, float4* d_f32, unsigned long long* ctr) {
    if ((need & ~F0) == 0u)
        hipLaunchKernelGGL((ray_kernel<MODE, CULL, F0>), grid, block, 0, st, k, sv, cl, d_rgba, d_f32, ctr);
    else if ((need & ~F1) == 0u)
        hipLaunchKernelGGL((ray_kernel<MODE, CULL, F1>), grid, block, 0, st, k, sv, cl, d_rgba, d_f32, ctr);
    else if ((need & ~F2) == 0u)
        hipLaunchKernelGGL((ray_kernel<MODE, CULL, F2>), grid, block, 0, st, k, sv, cl, d_rgba, d_f32, ctr);
    else
        hipLaunchKernelGGL((ray_kernel<MODE, CULL, kFeatAll>), grid, block, 0, st, k, sv, cl, d_rgba, d_f32, ctr);
}

// Launch plan `L` (L.k.nframes frames) on `st`; the cached scene is the plan's.
rrte_status issue_launch(rrte_ctx* c, LaunchPlan& L, uint32_t* d_rgba, float4* d_f32, hipStream_t st) {
    if (L.gy == 0) return RRTE_OK;
    HostSection hsa(c);
    Cull cl{L.cull ? c->d_bounds : nullptr, L.num_prims};
    JitKernel* jk = jit_kernel_for(c, L.mode, L.cull, L.single);
    c->stats.jit_active = jk ? (jk->topology ? 2u : 1u) : 0u;
    // 64-thread workgroups: (tile column, frame, tile row or slot row), KParams::hot
    const bool profile = plan_tile_order(c, L, jk ? (const void*)jk->fn : nullptr, st);
    c->stats.hot_tiles = L.k.hot_n;
    if (c->sb_cur >= 0) {  // the launch reads the current scene version: after its upload, tracked until retired
        rrte_ctx::SceneBuf& B = c->sb[c->sb_cur];
        if (std::find(B.ordered.begin(), B.ordered.end(), st) == B.ordered.end()) {
            HIPCHK(c, ev_wait(c, st, B.ev_up, "wait scene upload"));
            B.ordered.push_back(st);
        }
        B.ret.use(st);
    }
    c->launched.use(st);
    if (c->ctr_pending && st != c->stream &&
        std::find(c->ctr_ordered.begin(), c->ctr_ordered.end(), st) == c->ctr_ordered.end()) {
        HIPCHK(c, ev_wait(c, st, c->ev_ctr[c->ctr_slot], "wait counter snapshot"));
        c->ctr_ordered.push_back(st);
    }
    const dim3 grid(L.gx, L.k.nframes, L.gy), block(kBlockThreads);
    trace_rec(c, profile ? "launch ray (profiled)" : "launch ray", st, nullptr, L.k.nframes, L.k.rows);
    if (jk) {
        unsigned long long* ctr = c->d_counters;
        MeshView mv = c->mesh_view;
        SceneValues vals{c->d_prims, c->d_mats, c->d_lights, c->d_nodes};  // read by topology kernels
        void* args[] = {&L.k, &cl, &mv, &d_rgba, &d_f32, &ctr, &vals};
        if (c->hpa_cur) hsa.lap(13);
        HostSection hs(c);
        if (c->env_wg256)
            HIPCHK(c, hipModuleLaunchKernel(jk->fn, (L.k.width + 15) / 16, (L.k.rows + 15) / 16, L.k.nframes, 256, 1, 1,
                                            0, st, args, nullptr));
        else
            HIPCHK(c, hipModuleLaunchKernel(jk->fn, grid.x, grid.y, grid.z, kBlockThreads, 1, 1, 0, st, args, nullptr));
        hs.lap(c->hpa_cur ? 14 : 8);
        return finish_tile_order(c, L, profile, st);
    }
    SceneView sv{c->d_prims, c->d_mats, c->d_lights, c->d_nodes, L.num_prims, L.num_lights, L.num_materials,
                 c->mesh_view};
    const KParams& k = L.k;
    const uint32_t need = c->env_generic_all ? kFeatAll : c->scene_feat;
    if (L.mode == RRTE_MODE_REFCOMPAT)
        launch_generic<RRTE_MODE_REFCOMPAT, false, 0u, kFeatAnalytic, kFeatSdf>(need, grid, block, st, k, sv, cl, d_rgba,
                                                                             d_f32, c->d_counters);
    else if (L.cull)
        launch_generic<RRTE_MODE_LAMBERT_SHADOW, true, kFeatSdf, kFeatSdf | kFeatDeform, kFeatSdf | kFeatAnalytic>(
            need, grid, block, st, k, sv, cl, d_rgba, d_f32, c->d_counters);
    else
        launch_generic<RRTE_MODE_LAMBERT_SHADOW, false, 0u, kFeatAnalytic, kFeatSdf>(need, grid, block, st, k, sv, cl,
                                                                                    d_rgba, d_f32, c->d_counters);
    HIPCHK(c, hipGetLastError());
    return finish_tile_order(c, L, profile, st);
}

rrte_status launch(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, uint32_t rows,
                   uint32_t* d_rgba, float4* d_f32, hipStream_t st, uint32_t internal_flags = 0u, uint32_t row0 = 0u,
                   int prof = 0, const BandMap* bm = nullptr) {
    if (rows == 0) return RRTE_OK;
    HostSection hs(c);
    LaunchPlan L = plan_launch(c, s, p, rows, internal_flags, row0, bm);
    if (c->hpa_cur) hs.lap(12);
    L.prof = prof;
    return issue_launch(c, L, d_rgba, d_f32, st);
}

unsigned long long* ctr_host(rrte_ctx* c, int slot) { return slot ? c->h_counters2 : c->h_counters; }
unsigned long long ctr_total(rrte_ctx* c, int slot) {
    const unsigned long long* h = ctr_host(c, slot);
    unsigned long long total = 0;
    for (uint32_t i = 0; i < kCounterShards; ++i) total += h[i * kCounterStride];
    return total;
}

// The last blocking frame's shadow-ray count into rrte_stats (waits for its counter copy).
rrte_status resolve_counters(rrte_ctx* c) {
    if (!c->ctr_pending) return RRTE_OK;
    HIPCHK(c, hipEventSynchronize(c->ev_ctr[c->ctr_slot]));
    const unsigned long long total = ctr_total(c, c->ctr_slot);
    c->stats.shadow_rays = total - c->shadow_base;
    c->shadow_base = total;
    c->ctr_pending = false;
    return RRTE_OK;
}

// Wait for `ev` by polling (a blocking wait wakes the host several us after the device signals):
// at most ~2 ms of polling, then a blocking wait.
rrte_status spin_wait(rrte_ctx* c, hipEvent_t ev) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return RRTE_OK;
        if (e != hipErrorNotReady) HIPCHK(c, e);
        if ((spin & 63u) == 63u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
            HIPCHK(c, hipEventSynchronize(ev));
            return RRTE_OK;
        }
    }
}

// Read back the device counters and close the frame's statistics.  `deferred` (the blocking
// single-context frame): return once the frame's work on the context's stream is complete; the
// counter copy queued behind it is folded in by resolve_counters when the statistics are read.
rrte_status finish_frame(rrte_ctx* c, bool deferred = false) {
    // the slot the pending copy does not use (that copy precedes this one on the stream)
    const int slot = c->ctr_pending ? 1 - c->ctr_slot : 0;
    if (deferred) HIPCHK(c, hipEventRecord(c->ev_done, c->stream));
    HIPCHK(c, hipMemcpyAsync(ctr_host(c, slot), c->d_counters, kCounterBytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(c->ev_ctr[slot], c->stream));
    rrte_status r = deferred ? spin_wait(c, c->ev_done) : RRTE_OK;
    if (r != RRTE_OK) return r;
    trace_rec(c, "frame complete (host)", c->stream, nullptr);
    if (!deferred) HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->ctr_pending) {
        // (complete: it precedes this frame on the stream) the previous frame's counts, never read,
        // become the base of this one's
        c->shadow_base = ctr_total(c, c->ctr_slot);
        c->ctr_pending = false;
    }
    c->ctr_slot = slot;
    c->ctr_pending = true;
    c->ctr_ordered.clear();
    if (!deferred && (r = resolve_counters(c)) != RRTE_OK) return r;
    if (c->pending_kernel_timing) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) c->stats.kernel_ms = ms;
        c->pending_kernel_timing = false;
    }
    c->stats.primary_rays = c->pending_primary;
    return RRTE_OK;
}

// The blocking drop-in path into a host RGBA8 buffer (Raytracer::render, raytracer.rs:45-89): the
// frame renders as `n` row chunks (multiples of 16 rows, so camera-culling tiles never straddle two
// chunks), each launched on a stream of its own so they run together as one frame would, each in its
// own measured-cost tile order (tile-profile slot 1 + i).  Each chunk's D2H copy starts on the copy
// stream as soon as that chunk's kernel has completed -- the kernel boundary orders its stores, no
// fences -- so the 8.3 MB PCIe copy (~150 us at ~55 GB/s) overlaps the rest of the render instead of
// following all of it.  Copies run top to bottom.
rrte_status render_chunked(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, uint8_t* out8,
                           uint32_t n) {
    const uint32_t W = p->width, H = p->height;
    const uint32_t rows = (((H + n - 1) / n) + 15u) & ~15u;
    n = (H + rows - 1) / rows;
    for (uint32_t i = 0; i < n; ++i) {
        if (!c->bnd_stream[i]) HIPCHK(c, hipStreamCreateWithFlags(&c->bnd_stream[i], hipStreamNonBlocking));
        if (!c->ev_bchunk[i]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_bchunk[i], hipEventDisableTiming));
    }
    if (!c->bnd_copy) HIPCHK(c, hipStreamCreateWithFlags(&c->bnd_copy, hipStreamNonBlocking));
    if (!c->ev_bcopy) HIPCHK(c, hipEventCreateWithFlags(&c->ev_bcopy, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));  // after the work already queued on the context's stream
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t r0 = i * rows, nr = std::min(rows, H - r0);
        HIPCHK(c, hipStreamWaitEvent(c->bnd_stream[i], c->ev0, 0));
        rrte_status r = launch(c, s, p, nr, c->d_rgba + (size_t)r0 * W, nullptr, c->bnd_stream[i], 0u, r0, 1 + (int)i);
        if (r != RRTE_OK) return r;
        HIPCHK(c, hipEventRecord(c->ev_bchunk[i], c->bnd_stream[i]));
    }
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t r0 = i * rows, nr = std::min(rows, H - r0);
        HIPCHK(c, hipStreamWaitEvent(c->bnd_copy, c->ev_bchunk[i], 0));
        HIPCHK(c, hipMemcpyAsync(out8 + (size_t)r0 * W * 4, c->d_rgba + (size_t)r0 * W, (size_t)nr * W * 4,
                                 hipMemcpyDeviceToHost, c->bnd_copy));
    }
    HIPCHK(c, hipEventRecord(c->ev_bcopy, c->bnd_copy));
    // the context's stream: every chunk (ev1: the render's end, rrte_stats.kernel_ms), then the copies
    for (uint32_t i = 0; i < n; ++i) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_bchunk[i], 0));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_bcopy, 0));
    return RRTE_OK;
}

// The device address of pinned host memory [host, host + bytes) -- hipHostMalloc'd, or registered
// (rrte_hip_host_register, hipHostRegister) -- or nullptr for pageable memory.  The whole range must
// lie in one pinned allocation.
uint32_t* pinned_device_ptr(void* host, size_t bytes) {
    hipPointerAttribute_t a{}, b{};
    if (hipPointerGetAttributes(&a, host) != hipSuccess) {
        (void)hipGetLastError();  // (pageable memory: not an error of this call)
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
    uint8_t* last = static_cast<uint8_t*>(host) + bytes - 1;
    if (hipPointerGetAttributes(&b, last) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (b.type != hipMemoryTypeHost || static_cast<uint8_t*>(b.devicePointer) != static_cast<uint8_t*>(a.devicePointer) + bytes - 1)
        return nullptr;
    return static_cast<uint32_t*>(a.devicePointer);
}

// RRTE_DUMP_SCENE (diagnostics): the frame's scene and parameters, as given, into the dump file
// before anything else happens to them (rrte_hip_scene_dump; replayable on the oracle or the device).
void dump_if_asked(const rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p) {
    if (!c->dump_path.empty() && s && p) (void)rrte_hip_scene_dump(s, p, c->dump_path.c_str());
}

rrte_status render_common(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, uint8_t* out8,
                          float* outf) {
    dump_if_asked(c, s, p);
    rrte_status r = validate(c, s, p);
    if (r != RRTE_OK) return r;
    HIPCHK(c, hipSetDevice(c->device));
    double up = 0.0;
    if ((r = upload_scene(c, s, c->stream, &up)) != RRTE_OK) return r;
    const size_t npix = (size_t)p->width * p->height;
    if ((r = ensure(c, c->d_rgba, c->cap_rgba, npix)) != RRTE_OK) return r;
    if (outf && (r = ensure(c, c->d_f32, c->cap_f32, npix)) != RRTE_OK) return r;
    // single-context render: all rows, no band mapping
    const int nr = c->nranks, rk = c->rank;
    c->nranks = 1;
    c->rank = 0;
    c->jit_stream = false;  // (one blocking frame: the latency flavour of the specialised kernel)
    // pinned caller buffer: the kernel writes the frame into it directly (no D2H copy afterwards)
    uint32_t* zc = out8 && !outf && c->env_bnd_zerocopy ? pinned_device_ptr(out8, npix * 4) : nullptr;
    const bool chunked = !zc && out8 && !outf && c->bnd_chunks > 1 && p->height >= 32u && !(c->env_debug & ~4u);  // (bit 2, the index check, keeps every path)
    if (chunked) {
        r = render_chunked(c, s, p, out8, (uint32_t)c->bnd_chunks);
    } else {
        HIPCHK(c, hipEventRecord(c->ev0, c->stream));
        if (zc) c->tile_shift = c->zc_tile_shift;  // whole 128-B lines per wave across PCIe
        r = launch(c, s, p, p->height, zc ? zc : c->d_rgba, outf ? c->d_f32 : nullptr, c->stream,
                   zc && c->env_zc_system_store ? kFlagHostStore : 0u, 0u, zc ? rrte_ctx::kZcProf : 0);
        c->tile_shift = 3;
        if (r == RRTE_OK) r = hipEventRecord(c->ev1, c->stream) == hipSuccess ? RRTE_OK : RRTE_HIP_ERROR;
    }
    c->nranks = nr;
    c->rank = rk;
    c->jit_stream = true;
    if (r != RRTE_OK) return r;
    c->pending_kernel_timing = true;
    c->pending_primary = (uint64_t)npix * p->samples_per_pixel;
    c->stats.upload_ms = up;
    c->stats.gather_ms = 0.0;
    if (out8 && !chunked && !zc) HIPCHK(c, hipMemcpyAsync(out8, c->d_rgba, npix * 4, hipMemcpyDeviceToHost, c->stream));
    if (outf) HIPCHK(c, hipMemcpyAsync(outf, c->d_f32, npix * 16, hipMemcpyDeviceToHost, c->stream));
    if ((r = finish_frame(c, true)) != RRTE_OK) return r;
    c->stats.frames++;
    return RRTE_OK;
}

}  // namespace

// ---------------------------------------------------------- rrte_hip_fpcheck
// Bit-exactness sweeps of device_scene.hpp's short correctly rounded sequences against the
// compiler's full ones.  A mismatch count is accumulated per wave (ballot + popcount).
__device__ __forceinline__ bool fp_same(float a, float b) {
    return (a != a && b != b) || __float_as_uint(a) == __float_as_uint(b);
}
__device__ __forceinline__ void fp_count(bool bad, unsigned long long* out) {
    const unsigned long long m = __ballot(bad);
    if (m && (threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)__popcll(m));
}
__global__ __launch_bounds__(256) void fpcheck_unary_kernel(int kind, uint64_t x0, uint64_t n,
                                                            unsigned long long* out) {
    // thread t of the launch checks patterns x0 + t + k * (launch threads), k < 64
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < stride * 64; i += stride) {
        const bool in = i < n;
        const float x = __uint_as_float((uint32_t)(x0 + (in ? i : 0)));
        bool bad;
        if (kind == RRTE_FPCHECK_SQRT) bad = !fp_same(sqrt_rn_guarded(x), __builtin_sqrtf(x));
        else if (kind == RRTE_FPCHECK_SQRT_BF) bad = !fp_same(sqrt_rn_branchfree(x), __builtin_sqrtf(x));
        else if (kind == RRTE_FPCHECK_RCP) bad = !fp_same(rcp_rn(x), 1.0f / x);
        else if (kind == RRTE_FPCHECK_GAMMA_U8) bad = gamma22_u8(x) != to_u8(rclamp(powf(x, kInvGamma22)));
        else bad = !fp_same(__builtin_amdgcn_sqrtf(x), __builtin_sqrtf(x));
        fp_count(in && bad, out);
    }
}
__global__ __launch_bounds__(256) void fpcheck_div_kernel(uint32_t b0, unsigned long long* out) {
    const float b = __uint_as_float(0x3f800000u | (b0 + blockIdx.x));
    const float y = rcp_rn(b);
    for (uint32_t am = threadIdx.x; am < (1u << 23); am += blockDim.x) {
        const float a = __uint_as_float(0x3f800000u | am);
        fp_count(!fp_same(div_by_rcp(a, b, y), a / b), out);
    }
}

extern "C" {

uint32_t rrte_hip_abi_version(void) { return RRTE_ABI_VERSION; }

rrte_status rrte_hip_create(int device, rrte_ctx** out) {
    if (!out) return RRTE_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return RRTE_NO_DEVICE;
    if (device < 0 || device >= n) return RRTE_NO_DEVICE;
    rrte_ctx* c = new (std::nothrow) rrte_ctx();
    if (!c) return RRTE_HIP_ERROR;
    c->device = device;
    if (const char* j = getenv("RRTE_JIT")) c->jit_mode = (int)strtol(j, nullptr, 0);
    if (const char* d = getenv("RRTE_DEBUG")) c->env_debug = (uint32_t)strtoul(d, nullptr, 0);
    c->env_cull = env_cull_setting();
    if (const char* t = getenv("RRTE_TILE_CULL")) c->env_tile_cull = t[0] != '0';
    if (const char* g = getenv("RRTE_FORCE_GATHER")) c->env_force_gather = g[0] == '1';
    if (const char* g = getenv("RRTE_HOST_PROFILE")) c->host_prof = g[0] == '1';
    if (const char* g = getenv("RRTE_TRACE")) c->trace = g[0] == '1';
    if (const char* g = getenv("RRTE_DIAG_SKIP")) c->env_diag_skip = (uint32_t)strtoul(g, nullptr, 0);
    if (const char* g = getenv("RRTE_GATHER_RGB24")) c->env_gather_rgba = g[0] == '0';
    c->env_guard_leaves = env_guard_setting();
    if (const char* g = getenv("RRTE_COMM_TIMEOUT_MS")) c->comm_timeout_ms = std::max<uint32_t>(1u, (uint32_t)strtoul(g, nullptr, 0));
    if (const char* g = getenv("RRTE_FAULT_STALL_GATHER")) c->fault_stall_at = strtoull(g, nullptr, 0);
    if (const char* g = getenv("RRTE_BATCH_SLABS"); g && *g)
        c->batch_slabs = std::max(1, std::min(rrte_ctx::kBatchSlabs, (int)strtol(g, nullptr, 0)));
    if (const char* g = getenv("RRTE_GATHER_SELF")) c->env_gather_self = g[0] == '1';
    if (const char* g = getenv("RRTE_BAND_SKY")) c->env_band_sky = g[0] != '0';
    if (const char* g = getenv("RRTE_COMM_PRIORITY")) c->env_comm_priority = g[0] != '0';
    if (const char* g = getenv("RRTE_WG64")) c->env_wg256 = g[0] == '0';
    if (const char* g = getenv("RRTE_GENERIC_ALL")) c->env_generic_all = g[0] == '1';
    if (const char* g = getenv("RRTE_GUARD_POLICY"); g && *g) c->env_guard_policy = std::min(2, std::max(0, atoi(g)));
    if (const char* g = getenv("RRTE_BATCH_LAUNCH")) c->env_batch_launch = g[0] != '0';
    if (const char* g = getenv("RRTE_BND_ZEROCOPY")) c->env_bnd_zerocopy = g[0] != '0';
    if (const char* g = getenv("RRTE_ZC_TILE_SHIFT"))
        c->zc_tile_shift = std::max(3u, std::min(6u, (uint32_t)strtoul(g, nullptr, 0)));
    if (const char* g = getenv("RRTE_ZC_SYSTEM_STORE")) c->env_zc_system_store = g[0] != '0';
    if (const char* g = getenv("RRTE_NOCOMM_WAIT_MS")) c->env_nocomm_wait_ms = (uint32_t)strtoul(g, nullptr, 0);
    if (const char* g = getenv("RRTE_TILE_ORDER")) {
        c->env_tile_order = g[0] != '0';
        c->env_tile_order_fixed = g[0] == '2';  // 0 image order, 2 fixed permutation (tests), else measured (default)
    }
    if (const char* g = getenv("RRTE_TEST_RECYCLE")) c->env_test_recycle = g[0] == '1';
    if (const char* g = getenv("RRTE_FAULT_BAD_SLOT")) c->env_fault_bad_slot = (g[0] == '1' || g[0] == '2') ? g[0] - '0' : 0;
    if (const char* g = getenv("RRTE_DUMP_SCENE"); g && *g) c->dump_path = g;
    if (const char* g = getenv("RRTE_BND_CHUNKS"); g && *g)
        c->bnd_chunks = std::max(1, std::min(rrte_ctx::kBndChunksMax, (int)strtol(g, nullptr, 0)));
    if (const char* t = getenv("RRTE_JIT_TOPO"); t && *t) c->env_jit_topo = (int)strtol(t, nullptr, 0);
    if (const char* e = getenv("RRTE_EMULATE_PEERS")) {
        const int n = (int)strtol(e, nullptr, 0);
        if (n > 1) c->emu_peers = n;
    }
    if (const char* e = getenv("RRTE_EMULATE_RANK")) {
        int n = 0, r = 0;
        if (sscanf(e, "%d:%d", &n, &r) == 2 && n > 1 && r >= 0 && r < n) {
            c->emu_nranks = n;
            c->emu_rank = r;
        }
    }
    auto bail = [&](hipError_t e) {
        (void)e;
        rrte_hip_destroy(c);
        return RRTE_HIP_ERROR;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return bail(e);
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return bail(e);
    if ((e = hipEventCreate(&c->ev0)) != hipSuccess) return bail(e);
    if ((e = hipEventCreate(&c->ev1)) != hipSuccess) return bail(e);
    if ((e = hipEventCreate(&c->ev2)) != hipSuccess) return bail(e);
    if ((e = hipMalloc(reinterpret_cast<void**>(&c->d_counters), kCounterBytes)) != hipSuccess) return bail(e);
    // (on the context's stream: its first operation sets up its hardware queue, here and not in a frame)
    if ((e = hipMemsetAsync(c->d_counters, 0, kCounterBytes, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return bail(e);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&c->h_counters), kCounterBytes, hipHostMallocDefault)) != hipSuccess) return bail(e);
    memset(c->h_counters, 0, kCounterBytes);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&c->h_counters2), kCounterBytes, hipHostMallocDefault)) != hipSuccess) return bail(e);
    memset(c->h_counters2, 0, kCounterBytes);
    for (hipEvent_t& ev : c->ev_ctr)
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return bail(e);
    if ((e = hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming)) != hipSuccess) return bail(e);
    // the upload stream, and a first copy of a tile list's size class through it: the runtime sets up
    // what such a copy needs at its first use (7-8 ms measured, inside the first frame of a new launch
    // shape: profiles/r06_engine_loop_trace.log) -- here rather than in a frame
    if ((e = hipStreamCreateWithFlags(&c->upload_stream, hipStreamNonBlocking)) != hipSuccess) return bail(e);
    {
        // the library's code object (every generic kernel): the runtime loads it at a kernel's first
        // use -- ~20 ms inside the first frame otherwise (profiles/r06_engine_loop_trace_after.log)
        hipFuncAttributes fa;
        if ((e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&scene_records_check))) != hipSuccess)
            return bail(e);
    }
    {
        constexpr size_t kWarm = 129600;  // a 1080p frame's list (32400 slots)
        // (the buffers are freed with the context: a free here could wait for other contexts' frames)
        if ((e = hipHostMalloc(&c->h_warm, kWarm, hipHostMallocDefault)) != hipSuccess) return bail(e);
        memset(c->h_warm, 0, kWarm);
        // (and the way back on the context's stream: a frame's tile-profile copy is a D2H of that size)
        if ((e = hipMalloc(&c->d_warm, kWarm)) != hipSuccess ||
            (e = hipMemcpyAsync(c->d_warm, c->h_warm, kWarm, hipMemcpyHostToDevice, c->upload_stream)) != hipSuccess ||
            (e = hipStreamSynchronize(c->upload_stream)) != hipSuccess ||
            (e = hipMemcpyAsync(c->h_warm, c->d_warm, kWarm, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
            (e = hipStreamSynchronize(c->stream)) != hipSuccess)
            return bail(e);
    }
    if (c->fault_stall_at) {
        if ((e = hipHostMalloc(reinterpret_cast<void**>(&c->h_stall), 64, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
            return bail(e);
        *c->h_stall = 1u;
    }
    *out = c;
    return RRTE_OK;
}

void rrte_hip_destroy(rrte_ctx* c) {
    if (!c) return;
    if (c->host_prof && c->hp_frames) {
        static const char* names[9] = {"validate", "upload_check", "slab_setup", "render_launch", "event_chain",
                                       "ncclGather", "deinterleave", "event_record", "(of render_launch: the launch call)"};
        fprintf(stderr, "rrte host profile (%llu gather frames, us/frame):", (unsigned long long)c->hp_frames);
        for (int i = 0; i < 9; ++i) fprintf(stderr, " %s %.2f", names[i], c->hp[i] / (double)c->hp_frames);
        fprintf(stderr, "\n");
    }
    if (c->host_prof && c->hpa_frames) {
        static const char* names[5] = {"validate", "scene_check", "plan", "tile_order+jit", "launch_call"};
        fprintf(stderr, "rrte host profile (%llu async frames, us/frame):", (unsigned long long)c->hpa_frames);
        for (int i = 0; i < 5; ++i) fprintf(stderr, " %s %.2f", names[i], c->hp[10 + i] / (double)c->hpa_frames);
        fprintf(stderr, "\n");
    }
    if (c->host_prof && c->hpu_n) {
        static const char* names[9] = {"lower", "mesh_bvh", "csg_guards", "topology", "version_wait", "staging",
                                       "copy_call", "event_record", "bookkeeping"};
        fprintf(stderr, "rrte host profile (%llu scene uploads, us/upload):", (unsigned long long)c->hpu_n);
        for (int i = 0; i < 9; ++i) fprintf(stderr, " %s %.2f", names[i], c->hpu[i] / (double)c->hpu_n);
        fprintf(stderr, "\n");
    }
    if (c->trace) {
        for (const auto& t : c->trace_log)
            fprintf(stderr, "rrte trace %12.1f us  %-34s stream %p event %p  %u %u\n", t.us, t.what, t.st, t.ev, t.a, t.b);
    }
    (void)hipSetDevice(c->device);
    if (c->h_stall) __hip_atomic_store(c->h_stall, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // injected stall
    // gathers first, bounded (a dead peer aborts the communicator instead of hanging here); then the
    // frames that may still run on caller streams
    if (c->comm && wait_bounded(c) != RRTE_OK) c->comm = nullptr;  // (comm_abort has aborted it)
    (void)hipDeviceSynchronize();
    if (c->comm) ncclCommDestroy(c->comm);
    for (const auto& hr : c->host_regs) (void)hipHostUnregister(hr.p);
    c->jit_pending.clear();  // joins background compiles
    for (auto& kv : c->jit_cache) jit_release(kv.second);
    for (auto& B : c->sb) {
        if (B.d_buf) (void)hipFree(B.d_buf);
        if (B.h_stage) (void)hipHostFree(B.h_stage);
        if (B.ev_up) (void)hipEventDestroy(B.ev_up);
        destroy_events(B.ret);
    }
    void* bufs[] = {c->d_rgba, c->d_f32, c->d_counters, c->d_gather, c->d_full};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (void* b : c->graveyard)
        if (b) (void)hipFree(b);
    destroy_events(c->launched);
    for (uint32_t* b : c->d_slab)
        if (b) (void)hipFree(b);
    if (c->h_counters) (void)hipHostFree(c->h_counters);
    if (c->h_counters2) (void)hipHostFree(c->h_counters2);
    if (c->h_warm) (void)hipHostFree(c->h_warm);
    if (c->d_warm) (void)hipFree(c->d_warm);
    for (hipEvent_t e : c->ev_ctr)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    if (c->h_stall) (void)hipHostFree(c->h_stall);
    for (auto& tp : c->tprof) {
        if (tp.working) tp.work.wait();
        if (tp.d_cost) (void)hipFree(tp.d_cost);
        if (tp.h_cost) (void)hipHostFree(tp.h_cost);
        if (tp.ev) (void)hipEventDestroy(tp.ev);
        for (int i = 0; i < rrte_ctx::TileProfile::kVersions; ++i) {
            if (tp.d_list[i]) (void)hipFree(tp.d_list[i]);
            destroy_events(tp.ret[i]);
        }
        if (tp.h_arena) (void)hipHostFree(tp.h_arena);
        for (hipEvent_t e : tp.ev_up)
            if (e) (void)hipEventDestroy(e);
    }
    for (int i = 0; i < rrte_ctx::kBndChunksMax; ++i) {
        if (c->bnd_stream[i]) (void)hipStreamDestroy(c->bnd_stream[i]);
        if (c->ev_bchunk[i]) (void)hipEventDestroy(c->ev_bchunk[i]);
    }
    if (c->bnd_copy) (void)hipStreamDestroy(c->bnd_copy);
    if (c->ev_bcopy) (void)hipEventDestroy(c->ev_bcopy);
    if (c->upload_stream) (void)hipStreamDestroy(c->upload_stream);
    for (hipEvent_t e : c->ev_poll)
        if (e) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    for (hipEvent_t e : c->ev_gath)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_batch)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_render)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->batch.ev_src)
        if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < rrte_ctx::kBatchSlabs; ++i) {
        if (c->d_bsend[i]) (void)hipFree(c->d_bsend[i]);
        if (c->d_brecv[i]) (void)hipFree(c->d_brecv[i]);
        if (c->render_stream[i]) (void)hipStreamDestroy(c->render_stream[i]);
    }
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* rrte_hip_last_error(const rrte_ctx* c) { return c ? c->err.c_str() : "null context"; }

rrte_status rrte_hip_render(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, uint8_t* out) {
    if (!c) return RRTE_INVALID_ARG;
    if (!out) return fail(c, RRTE_INVALID_ARG, "null output buffer");
    trace_rec(c, "render: enter", nullptr, nullptr);
    return render_common(c, s, p, out, nullptr);
}

rrte_status rrte_hip_render_f32(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, uint8_t* out8,
                                float* outf) {
    if (!c) return RRTE_INVALID_ARG;
    return render_common(c, s, p, out8, outf);
}

rrte_status rrte_hip_render_async(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, void* d_rgba,
                                  void* d_f32, void* stream) {
    if (!c) return RRTE_INVALID_ARG;
    dump_if_asked(c, s, p);
    HostSection hs(c);
    rrte_status r = validate(c, s, p);
    if (r != RRTE_OK) return r;
    hs.lap(10);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : c->stream;
    double up = 0.0;
    if ((r = upload_scene(c, s, st, &up)) != RRTE_OK) return r;
    hs.lap(11);
    c->hpa_cur = true;
    const int nr = c->nranks, rk = c->rank;
    uint32_t rows = p->height;
    rrte_render_params pe = *p;
    BandMap bm{0u, 1u, 0u, 1u, 1u};
    if (c->emu_nranks > 1) {  // diagnostic: exactly one rank's share of a multi-GPU frame, packed
        c->nranks = c->emu_nranks;
        c->rank = c->emu_rank;
        pe.band_rows = p->band_rows ? p->band_rows : 16;
        bm = frame_band_map(c, s, &pe, 0, &rows);
    } else {
        c->nranks = 1;
        c->rank = 0;
    }
    r = launch(c, s, &pe, rows, static_cast<uint32_t*>(d_rgba), static_cast<float4*>(d_f32), st, 0u, 0u, 0, &bm);
    c->hpa_cur = false;
    c->nranks = nr;
    c->rank = rk;
    if (r != RRTE_OK) return r;
    c->hpa_frames += c->host_prof;
    c->pending_primary = (uint64_t)p->width * rows * p->samples_per_pixel;
    c->stats.upload_ms = up;
    c->stats.frames++;
    return RRTE_OK;
}

rrte_status rrte_hip_synchronize(rrte_ctx* c) {
    if (!c) return RRTE_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    // local: an open gather batch is rendered but stays open (its gather is collective: rrte_hip_flush)
    rrte_status r = render_batch(c, false);
    if (r != RRTE_OK) return r;
    if ((r = wait_bounded(c)) != RRTE_OK) return r;
    // every stream that launched a frame (bounded: a frame may sit behind a gather), then the device
    if ((r = retire(c, c->launched)) != RRTE_OK || (r = wait_retired(c, c->launched)) != RRTE_OK) return r;
    HIPCHK(c, hipDeviceSynchronize());
    // idle: buffers replaced while frames were in flight can go, and every retired version is free
    for (void* b : c->graveyard)
        if (b) (void)hipFree(b);
    c->graveyard.clear();
    return finish_frame(c);
}

rrte_status rrte_hip_check_word(rrte_ctx* c, uint64_t* word) {
    if (!c || !word) return RRTE_INVALID_ARG;
    rrte_status r = rrte_hip_synchronize(c);
    if (r != RRTE_OK) return r;
    unsigned long long w = 0;  // counters[1]: an unused word of shard 0 (ray_kernels.hpp launch_indices_ok)
    HIPCHK(c, hipMemcpy(&w, c->d_counters + 1, sizeof w, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemset(c->d_counters + 1, 0, sizeof w));
    *word = w;
    return RRTE_OK;
}

rrte_status rrte_hip_set_comm_timeout(rrte_ctx* c, uint32_t ms) {
    if (!c) return RRTE_INVALID_ARG;
    if (ms == 0) return fail(c, RRTE_INVALID_ARG, "comm timeout must be > 0 ms");
    c->comm_timeout_ms = ms;
    return RRTE_OK;
}

rrte_status rrte_hip_query(rrte_ctx* c, uint32_t* busy) {
    if (!c || !busy) return RRTE_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t ss[2 + rrte_ctx::kBatchSlabs] = {c->stream, c->comm_stream};
    for (int i = 0; i < rrte_ctx::kBatchSlabs; ++i) ss[2 + i] = c->render_stream[i];
    *busy = 0;
    for (hipStream_t s : ss) {
        if (!s) continue;
        const hipError_t e = hipStreamQuery(s);
        if (e == hipErrorNotReady) {
            *busy = 1;
            return RRTE_OK;
        }
        HIPCHK(c, e);
    }
    return RRTE_OK;
}

rrte_status rrte_hip_set_jit(rrte_ctx* c, int mode) {
    if (!c) return RRTE_INVALID_ARG;
    if (mode < RRTE_JIT_OFF || mode > RRTE_JIT_AUTO) return fail(c, RRTE_INVALID_ARG, "unknown JIT mode %d", mode);
    c->jit_mode = mode;
    return RRTE_OK;
}

rrte_status rrte_hip_stats(rrte_ctx* c, rrte_stats* out) {
    if (!c || !out) return RRTE_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    rrte_status r = resolve_counters(c);
    if (r != RRTE_OK) return r;
    *out = c->stats;
    return RRTE_OK;
}

rrte_status rrte_hip_sdf_guards(const rrte_sdf_node* in, uint32_t count, uint32_t min_leaves, rrte_sdf_node* out,
                                uint32_t* guards) {
    if ((count && (!in || !out)) || !guards) return RRTE_INVALID_ARG;
    if (count && !sdf_program_ok(in, count)) return RRTE_UNSUPPORTED_PRIM;
    if (count) memmove(out, in, sizeof(rrte_sdf_node) * count);
    for (uint32_t i = 0; i < count; ++i) out[i].i[kGuardSlot] = 0u;
    *guards = min_leaves && count ? decorate_sdf_guards(out, count, min_leaves) : 0u;
    return RRTE_OK;
}

rrte_status rrte_hip_tile_order_plan(const uint32_t* costs, uint32_t tiles, uint32_t tiles_x, uint32_t* slots,
                                     uint32_t cap, uint32_t* n_slots) {
    if (!costs || !slots || !n_slots || tiles == 0 || tiles_x == 0 || tiles_x > 0xffffu || tiles / tiles_x > 0xffffu)
        return RRTE_INVALID_ARG;
    const std::vector<uint32_t> v = lpt_slots(costs, tiles, tiles_x);
    *n_slots = (uint32_t)v.size();
    if (v.size() > cap) return RRTE_INVALID_ARG;
    std::copy(v.begin(), v.end(), slots);
    return RRTE_OK;
}

rrte_status rrte_hip_build_id(char* out, size_t out_len) {
    if (!out || out_len < 33) return RRTE_INVALID_ARG;
    // the device code's identity: the embedded headers, every hiprtc option (RRTE_JIT_EXTRA_OPTS
    // included) and the hiprtc version -- the JIT cache key of an empty source
    snprintf(out, out_len, "%s", jit_cache_name(std::string(), nullptr).c_str());
    return RRTE_OK;
}

rrte_status rrte_hip_jit_cache_key(const char* source, const char* headers_override, char* out, size_t out_len) {
    if (!source || !out || out_len < 33) return RRTE_INVALID_ARG;
    snprintf(out, out_len, "%s", jit_cache_name(source, headers_override).c_str());
    return RRTE_OK;
}

rrte_status rrte_hip_jit_check(const rrte_scene_ir* s, int mode, char* log, size_t log_len) {
    if (!s || (s->num_prims && !s->prims) || (s->num_sdf_nodes && !s->sdf_nodes)) return RRTE_INVALID_ARG;
    std::vector<DPrim> prims;
    std::vector<DMaterial> mats;
    std::vector<DLight> lights;
    if ((s->num_mesh_indices && !s->mesh_indices) || (s->num_mesh_vertices && !s->mesh_vertices)) return RRTE_INVALID_ARG;
    lower_scene(s, prims, mats, lights);
    MeshData md;
    build_mesh_bvhs(s, prims.data(), md, nullptr);
    // RRTE_JIT_CHECK_MULTI=1: the multi-sample / multi-bounce variant (as the renderer picks it for
    // spp > 1 or max_depth > 1) instead of the straight-line one
    const char* mv = getenv("RRTE_JIT_CHECK_MULTI");
    const bool single = !(mv && mv[0] == '1');
    std::vector<rrte_sdf_node> nodes = decorate_scene_sdf(s, env_guard_setting());
    JitTopo topo;
    topology_of(prims, lights, nodes, topo);
    // RRTE_JIT_TOPO=1: the topology kernel instead of the full one
    const char* tv = getenv("RRTE_JIT_TOPO");
    const bool want_topo = tv && tv[0] == '1';
    std::string src = jit_source(prims.data(), (uint32_t)prims.size(), mats.data(), (uint32_t)mats.size(),
                                 lights.data(), (uint32_t)lights.size(), nodes.data(), s->num_sdf_nodes, mode,
                                 cull_policy(s, (uint32_t)mode, env_cull_setting()), single,
                                 want_topo ? &topo : nullptr);
    std::string msg;
    bool ok = jit_compile_only(src, msg);
    if (log && log_len) {
        snprintf(log, log_len, "%s", ok ? "" : msg.c_str());
    }
    return ok ? RRTE_OK : RRTE_HIP_ERROR;
}

rrte_status rrte_hip_fpcheck(int device, int kind, uint64_t lo, uint64_t hi, uint64_t* mismatches) {
    if (!mismatches || kind < RRTE_FPCHECK_SQRT || kind > RRTE_FPCHECK_SQRT_BF || lo > hi ||
        hi > (kind == RRTE_FPCHECK_DIV ? (1ull << 23) : (1ull << 32)))
        return RRTE_INVALID_ARG;
    if (hipSetDevice(device) != hipSuccess) return RRTE_HIP_ERROR;
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, sizeof(unsigned long long)) != hipSuccess) return RRTE_HIP_ERROR;
    bool ok = hipMemset(d, 0, sizeof(unsigned long long)) == hipSuccess;
    if (kind == RRTE_FPCHECK_DIV) {
        const uint64_t chunk = 1u << 14;  // b significands per launch (one workgroup each)
        for (uint64_t b0 = lo; ok && b0 < hi; b0 += chunk) {
            const uint32_t n = (uint32_t)std::min<uint64_t>(chunk, hi - b0);
            hipLaunchKernelGGL(fpcheck_div_kernel, dim3(n), dim3(256), 0, 0, (uint32_t)b0, d);
            ok = hipGetLastError() == hipSuccess;
        }
    } else {
        const uint64_t chunk = 1ull << 26;  // bit patterns per launch, 64 per thread
        for (uint64_t x0 = lo; ok && x0 < hi; x0 += chunk) {
            const uint64_t n = std::min<uint64_t>(chunk, hi - x0);
            hipLaunchKernelGGL(fpcheck_unary_kernel, dim3((uint32_t)((n + 16383) / 16384)), dim3(256), 0, 0, kind, x0,
                               n, d);
            ok = hipGetLastError() == hipSuccess;
        }
    }
    unsigned long long h = 0;
    ok = ok && hipDeviceSynchronize() == hipSuccess &&
         hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d);
    if (!ok) return RRTE_HIP_ERROR;
    *mismatches = h;
    return RRTE_OK;
}

uint32_t rrte_hip_band_rows_for_rank(uint32_t height, uint32_t band_rows, int nranks, int rank) {
    return rows_for_rank(height, band_rows, nranks, rank);
}

rrte_status rrte_hip_band_layout(const rrte_scene_ir* s, const rrte_render_params* p, int nranks, int root,
                                 uint32_t* sky_bands, uint32_t* root_bands, uint32_t* peer_bands) {
    if (!s || !p || !sky_bands || !root_bands || !peer_bands || nranks < 1 || root < 0 || root >= nranks) return RRTE_INVALID_ARG;
    if ((s->num_prims && !s->prims) || (s->num_mesh_indices && !s->mesh_indices) ||
        (s->num_mesh_vertices && !s->mesh_vertices))
        return RRTE_INVALID_ARG;
    rrte_render_params pp = *p;
    if (!pp.band_rows) pp.band_rows = 16;
    std::vector<DPrim> prims;
    std::vector<DMaterial> mats;
    std::vector<DLight> lights;
    std::vector<float4> bounds;
    lower_scene(s, prims, mats, lights, &bounds);
    MeshData md;
    build_mesh_bvhs(s, prims.data(), md, bounds.data());
    const char* g = getenv("RRTE_BAND_SKY");
    const BandMap m = band_layout(s->camera, bounds, s->num_prims, pp.width, pp.height, pp.band_rows, nranks, root,
                                  !(g && g[0] == '0'));
    *sky_bands = m.sky;
    *root_bands = m.root_bands;
    *peer_bands = m.peer_bands;
    return RRTE_OK;
}

uint32_t rrte_hip_band_rows_for_rank_ex(uint32_t height, uint32_t band_rows, int nranks, int rank, uint32_t sky_bands,
                                        uint32_t root_bands, uint32_t peer_bands) {
    if (root_bands > kMaxCycleBands || peer_bands < 1u || peer_bands > kMaxCycleBands ||
        (root_bands == 0u && sky_bands == 0u))
        return 0u;  // (outside the documented range)
    return rows_for_rank(height, band_rows, nranks, rank, sky_bands, root_bands, peer_bands);
}

rrte_status rrte_hip_comm_unique_id(uint8_t out_id[RRTE_UNIQUE_ID_BYTES]) {
    if (!out_id) return RRTE_INVALID_ARG;
    static_assert(sizeof(ncclUniqueId) == RRTE_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return RRTE_RCCL_ERROR;
    memcpy(out_id, &id, sizeof id);
    return RRTE_OK;
}

rrte_status rrte_hip_comm_init(rrte_ctx* c, int nranks, int rank, const uint8_t id_bytes[RRTE_UNIQUE_ID_BYTES]) {
    if (!c || !id_bytes || nranks < 1 || rank < 0 || rank >= nranks) return fail(c, RRTE_INVALID_ARG, "bad comm args");
    HIPCHK(c, hipSetDevice(c->device));
    // frames already accepted into an open batch are gathered on the old communicator first (every rank
    // re-initialises together, so this collective matches); then nothing of the old one may still run
    rrte_status fr = c->comm ? flush_batch(c) : RRTE_OK;
    c->batch.n = c->batch.nsrc = c->batch.rendered = 0;
    if (fr == RRTE_OK && c->comm) fr = wait_bounded(c);
    if (fr == RRTE_OK) {  // the frames on caller streams too (bounded)
        if ((fr = retire(c, c->launched)) == RRTE_OK) fr = wait_retired(c, c->launched);
    }
    if (c->comm) ncclCommDestroy(c->comm);
    c->comm = nullptr;
    c->last_gather_stream = nullptr;
    c->last_gather_ev = nullptr;
    c->comm_failed = false;
    c->comm_fail_msg.clear();
    c->gathers_issued = 0;
    if (fr != RRTE_OK) return fr;
    ncclUniqueId id;
    memcpy(&id, id_bytes, sizeof id);
    // Non-blocking initialisation, polled under the same timeout as every gather wait: a peer that
    // never joins surfaces as RRTE_RCCL_ERROR instead of a hang in ncclCommInitRank.  (Every later call
    // on the communicator may then return ncclInProgress: nccl_settle.)
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const ncclResult_t ir = ncclCommInitRankConfig(&c->comm, nranks, id, rank, &cfg);
    if (ir != ncclSuccess && ir != ncclInProgress) {
        if (c->comm) (void)ncclCommAbort(c->comm);
        c->comm = nullptr;
        return fail(c, RRTE_RCCL_ERROR, "ncclCommInitRankConfig failed: %s", ncclGetErrorString(ir));
    }
    if (rrte_status r = nccl_settle(c, ir, "ncclCommInitRankConfig"); r != RRTE_OK) {
        if (c->comm) (void)ncclCommAbort(c->comm);
        c->comm = nullptr;
        c->comm_failed = false;  // (no communicator: a later comm_init starts clean)
        return r;
    }
    c->nranks = nranks;
    c->rank = rank;
    c->comm_size = nranks;
    if (nranks == 1 && c->emu_peers > 1) {
        // RRTE_EMULATE_PEERS=N: the root of N ranks whose peers' shares it renders itself (render_peers)
        c->nranks = c->emu_peers;
        c->rank = 0;
    } else if (nranks == 1 && c->emu_nranks > 1) {
        // RRTE_EMULATE_RANK=N:R with a 1-rank communicator (diagnostic, one GPU): the gather path lays
        // frames out as rank R of N -- R's bands rendered into its slab slice, the 1-rank gather moving
        // that slice, and on rank 0 the de-interleave of all N slices (the other N-1 hold whatever the
        // receive buffer held) -- i.e. one rank's whole per-frame cost except the xGMI transfers.
        c->nranks = c->emu_nranks;
        c->rank = c->emu_rank;
    }
    return RRTE_OK;
}

// Gather slabs carry RGB24 (3 B/pixel, 25 % fewer bytes over xGMI) when every pixel's alpha byte
// is provably 255.  LAMBERT_SHADOW never lets a light touch alpha (ray_kernels.hpp, shade_lambert):
// a sample's alpha is the background's (miss), 1 (no material, max_depth 0) or 1 + (a*0.1)*0.1 for
// the material's albedo alpha a, and the pixel's is rclamp((1 + sum of sample alphas) * inv_spp)
// (the sum starts from BLACK, alpha 1).  With every sample alpha >= 0 (spp 1) or >= 1 (spp n > 1:
// the sum is then >= n + 1 and (n + 1) * RN(1/n) >= 1), the clamp gives 1.0 and to_u8 255.  The
// test is on signs only (no host arithmetic to mirror); NaN fails it.  Every rank decides from the
// same scene and parameters, so all agree on the slab format.  RRTE_GATHER_RGB24=0 forces RGBA8.
bool slab_rgb24(const rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p) {
    if (c->env_gather_rgba || (c->env_debug & ~4u) || p->mode != RRTE_MODE_LAMBERT_SHADOW) return false;
    const float thr = p->samples_per_pixel == 1 ? 0.0f : 1.0f;
    if (!(p->background[3] >= thr)) return false;
    for (uint32_t i = 0; i < s->num_materials; ++i)
        if (!(s->materials[i].albedo[3] >= 0.0f)) return false;
    return true;
}

// Issue the open batch (batched gather): the comm stream waits for its frames' renders, gathers all
// of them to the root in one ncclGather (each rank sends its frames' slices back to back) and
// de-interleaves every frame into its caller buffer.  Every rank holds the same open batch (same
// frames in the same order), so the collective matches.
// De-interleave `n` gathered frames (ray_kernels.hpp deinterleave_batch_kernel) on `st`.
static rrte_status deinterleave(rrte_ctx* c, hipStream_t st, const uint8_t* gathered, const DeinterleaveTargets& t,
                                uint32_t n, uint32_t width, uint32_t height, const BandMap& bm, bool rgb24,
                                size_t rank_stride, size_t frame_stride, uint32_t skip_rank = ~0u) {
    trace_rec(c, "launch expansion", st, nullptr, n, height);
    bool vec4 = width % 4u == 0;
    for (uint32_t j = 0; j < n; ++j) vec4 = vec4 && reinterpret_cast<uintptr_t>(t.full[j]) % 16u == 0;
    const uint32_t per = vec4 ? 1024u : 256u;  // pixels one workgroup moves per pass
    const dim3 dg(std::min((width + per - 1) / per, 8u), height, n), db(256);
    if (rgb24 && vec4)
        hipLaunchKernelGGL((deinterleave_batch_kernel<true, true>), dg, db, 0, st, gathered, t, width, bm, rank_stride, frame_stride, skip_rank);
    else if (rgb24)
        hipLaunchKernelGGL((deinterleave_batch_kernel<true, false>), dg, db, 0, st, gathered, t, width, bm, rank_stride, frame_stride, skip_rank);
    else if (vec4)
        hipLaunchKernelGGL((deinterleave_batch_kernel<false, true>), dg, db, 0, st, gathered, t, width, bm, rank_stride, frame_stride, skip_rank);
    else
        hipLaunchKernelGGL((deinterleave_batch_kernel<false, false>), dg, db, 0, st, gathered, t, width, bm, rank_stride, frame_stride, skip_rank);
    HIPCHK(c, hipGetLastError());
    return RRTE_OK;
}

// RRTE_EMULATE_PEERS (tests): render every peer's share of `n` frames -- peer q's bands under the plan's
// band partition, packed, in the plan's slab format (RGB24 or RGBA8) -- into its receive slot
// slab + q * rank_stride (frame j at + j * frame_stride), on `st`: the bytes a real peer would have
// sent with ncclSend for the same frames.  `base` is the root's plan of these frames.
static rrte_status render_peers(rrte_ctx* c, const LaunchPlan& base, const FrameCam* cams, uint32_t n, uint8_t* slab,
                                size_t rank_stride, size_t frame_stride, int root, hipStream_t st) {
    const BandMap bm{base.k.band_rows, (uint32_t)c->nranks, base.k.sky_bands, base.k.root_bands, base.k.peer_bands};
    for (int q = 0; q < c->nranks; ++q) {
        if (q == root) continue;
        LaunchPlan L = base;
        L.k.rank = (uint32_t)q;
        L.k.rows = rows_for_rank(base.k.height, bm.band_rows, c->nranks, q, bm.sky, bm.root_bands, bm.peer_bands);
        L.gy = tile_grid_rows(L.k, L.k.rows);
        L.k.out_image_rows = 0u;
        L.k.frame_stride = frame_stride;
        L.prof = 1 + (q - 1) % rrte_ctx::kBndChunksMax;  // (a tile profile per peer shape)
        for (uint32_t j0 = 0; j0 < n; j0 += kMaxLaunchFrames) {
            const uint32_t nf = std::min<uint32_t>(n - j0, kMaxLaunchFrames);
            memcpy(L.k.cam, cams + j0, nf * sizeof(FrameCam));
            L.k.nframes = nf;
            uint8_t* dst = slab + (size_t)q * rank_stride + (size_t)j0 * frame_stride;
            rrte_status r = issue_launch(c, L, reinterpret_cast<uint32_t*>(dst), nullptr, st);
            if (r != RRTE_OK) return r;
        }
    }
    return RRTE_OK;
}

// Launch the open batch's frames that have not been rendered yet ([rendered, n)) into its send slab on
// the slab's render stream, after the work queued on the frames' caller streams.  Local: no
// collective, so a rank may call it on its own (a scene change through a non-gather entry point,
// rrte_hip_synchronize) without desynchronising the ranks' gathers.
static rrte_status render_batch(rrte_ctx* c, bool at_flush) {
    rrte_ctx::Batch& b = c->batch;
    if (b.rendered >= b.n) return RRTE_OK;
    HostSection hs(c);
    const int k = c->bslot;
    (void)at_flush;
    // The root renders its own bands straight into each frame's caller buffer at their image rows
    // (RGBA8; FrameCam::out): nothing of the root's share is copied, gathered or expanded.  Peers
    // render into the send slab (packed rows, RGB24 when alpha is provably 255).
    uint8_t* base = b.in_place ? nullptr : c->d_bsend[k];
    hipStream_t rs = c->render_stream[k];
    // the renders follow the frames' caller streams (scene uploads, the callers' own prior work) and
    // the slab's previous batch (its gather reads the send slab)
    if (!(c->env_diag_skip & 4u))
        for (uint32_t i = 0; i < b.nsrc; ++i) {
            HIPCHK(c, ev_record(c, b.ev_src[i], b.src[i], "record src (render)"));
            HIPCHK(c, ev_wait(c, rs, b.ev_src[i], "render waits src"));
        }
    if (b.rendered == 0) HIPCHK(c, ev_wait(c, rs, c->ev_batch[k], "render waits slab's last exchange"));
    hs.lap(2);
    // a copy of the batch's plan: b.plan's fields before KParams::nframes are the batch-compatibility
    // key gather_frame compares every new frame with, identically on every rank, so they stay as
    // planned (the in-place root's RGBA8 flag is this launch's business only)
    LaunchPlan L = b.plan;
    if (b.in_place) L.k.flags &= ~kFlagSlabRgb24;
    for (uint32_t j0 = b.rendered; j0 < b.n; j0 += kMaxLaunchFrames) {
        const uint32_t nf = std::min<uint32_t>(b.n - j0, kMaxLaunchFrames);
        memcpy(L.k.cam, b.cam + j0, nf * sizeof(FrameCam));
        L.k.nframes = nf;
        L.k.frame_stride = b.slice;
        L.k.out_image_rows = b.in_place ? 1u : 0u;
        uint8_t* dst = b.in_place ? nullptr : base + (size_t)j0 * b.slice;
        rrte_status r = issue_launch(c, L, reinterpret_cast<uint32_t*>(dst), nullptr, rs);
        if (r != RRTE_OK) return r;
    }
    b.rendered = b.n;
    HIPCHK(c, ev_record(c, c->ev_render[k], rs, "record render done"));
    hs.lap(3);
    return RRTE_OK;
}

__global__ void noop_kernel() {}

// The stalled-peer stand-in of RRTE_FAULT_STALL_GATHER: spins on a host-written flag (vector atomic
// loads at system scope) with its own 5 s deadline on the 100 MHz wall clock, so it always ends.
__global__ void stall_kernel(const uint32_t* flag) {
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u &&
           wall_clock64() - t0 < 500000000ull) {
        __builtin_amdgcn_s_sleep(10);
    }
}

// Before a collective on `st`: count it, and enqueue the injected stall if this is the one.
static rrte_status before_collective(rrte_ctx* c, hipStream_t st) {
    ++c->gathers_issued;
    if (c->fault_stall_at && c->gathers_issued == c->fault_stall_at && c->h_stall) {
        __hip_atomic_store(c->h_stall, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        uint32_t* dflag = nullptr;
        HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), c->h_stall, 0));
        hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, st, dflag);
        HIPCHK(c, hipGetLastError());
        c->stall_armed = true;
        c->fault_stall_at = 0;  // one-shot
    }
    return RRTE_OK;
}

// A call on the non-blocking communicator returned `r`: ncclInProgress means RCCL is still setting the
// operation up (connections, the communicator itself), and the next call may only follow once the
// communicator's state has left ncclInProgress -- polled under comm_timeout_ms.
static rrte_status nccl_settle(rrte_ctx* c, ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return RRTE_OK;
    if (r != ncclInProgress) return fail(c, RRTE_RCCL_ERROR, "%s failed: %s", what, ncclGetErrorString(r));
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        ncclResult_t st = ncclInProgress;
        if (ncclCommGetAsyncError(c->comm, &st) != ncclSuccess)
            return fail(c, RRTE_RCCL_ERROR, "%s: ncclCommGetAsyncError failed", what);
        if (st == ncclSuccess) return RRTE_OK;
        if (st != ncclInProgress) return fail(c, RRTE_RCCL_ERROR, "%s failed: %s", what, ncclGetErrorString(st));
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(c->comm_timeout_ms))
            return fail(c, RRTE_RCCL_ERROR, "%s did not complete within %u ms (a peer never joined?)", what,
                        c->comm_timeout_ms);
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// A gather failed or did not finish in time: release any injected stall, give the queued work a short
// bounded chance to drain (so nothing of this communicator is still running when it is torn down),
// abort the communicator and fail every later gather call until rrte_hip_comm_init.
static rrte_status comm_abort(rrte_ctx* c, const char* why) {
    if (c->stall_armed && c->h_stall) __hip_atomic_store(c->h_stall, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    c->stall_armed = false;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        bool busy = false;
        for (hipEvent_t e : c->ev_poll)
            if (e && hipEventQuery(e) == hipErrorNotReady) busy = true;
        if (!busy || std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2000)) break;
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    if (c->comm) (void)ncclCommAbort(c->comm);
    c->comm = nullptr;
    c->comm_failed = true;
    c->comm_fail_msg = why;
    rrte_ctx::Batch& b = c->batch;
    b.n = b.nsrc = b.rendered = 0;
    c->last_gather_stream = nullptr;
    c->last_gather_ev = nullptr;
    return fail(c, RRTE_RCCL_ERROR, "%s; communicator aborted (call rrte_hip_comm_init again)", why);
}

// Bounded wait for events: polls them (and, while a communicator exists, ncclCommGetAsyncError)
// instead of blocking, so work that sits behind a gather that never completes -- a dead or stalled
// peer -- surfaces as RRTE_RCCL_ERROR after comm_timeout_ms (the communicator aborted) instead of a
// hang.  Without a communicator no gather can stall a frame (an aborted one's kernels are being torn
// down), so the wait lasts as long as the device needs up to RRTE_NOCOMM_WAIT_MS (default 10 minutes,
// far above any queue of frames; RRTE_HIP_ERROR after it so a hung or faulted kernel still returns;
// 0 = no limit).
static rrte_status poll_events(rrte_ctx* c, const hipEvent_t* ev, size_t n) {
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t limit_ms = c->comm ? c->comm_timeout_ms : c->env_nocomm_wait_ms;
    for (uint32_t spin = 0;; ++spin) {
        bool busy = false;
        for (size_t i = 0; i < n; ++i) {
            const hipError_t e = hipEventQuery(ev[i]);
            if (e == hipErrorNotReady) {
                busy = true;
                break;
            }
            HIPCHK(c, e);
        }
        if (!busy) return RRTE_OK;
        const bool late = std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(limit_ms);
        if (c->comm) {
            ncclResult_t ae = ncclSuccess;
            if (ncclCommGetAsyncError(c->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                char why[256];
                snprintf(why, sizeof why, "RCCL asynchronous error: %s", ncclGetErrorString(ae));
                return comm_abort(c, why);
            }
            if (late) {
                char why[256];
                snprintf(why, sizeof why, "gather did not complete within %u ms (stalled or dead peer?)", c->comm_timeout_ms);
                return comm_abort(c, why);
            }
        } else if (late && limit_ms) {
            return fail(c, RRTE_HIP_ERROR, "device work did not complete within %u ms", limit_ms);
        }
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// Bounded wait for the context's own streams and its last gather (poll_events).
static rrte_status wait_bounded(rrte_ctx* c) {
    constexpr int kPoll = 3 + rrte_ctx::kBatchSlabs;
    static_assert(sizeof(c->ev_poll) / sizeof(c->ev_poll[0]) == kPoll, "poll events");
    hipStream_t ss[kPoll] = {c->stream, c->comm_stream, c->last_gather_stream};
    for (int i = 0; i < rrte_ctx::kBatchSlabs; ++i) ss[3 + i] = c->render_stream[i];
    size_t n = 0;
    for (int i = 0; i < kPoll; ++i) {
        if (!ss[i]) continue;
        if (!c->ev_poll[n]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_poll[n], hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(c->ev_poll[n], ss[i]));
        ++n;
    }
    return poll_events(c, c->ev_poll, n);
}

// Close the open batch (collective: every rank holds the same open batch -- same frames in the same
// order -- so the ncclGather matches): render what is not rendered yet, then ONE ncclGather on the
// comm stream moves every frame's slices to the root, which de-interleaves each into its caller
// buffer.  Any failure resets the batch and aborts the communicator: a half-issued batch would leave
// the ranks' collectives out of step.
static rrte_status flush_batch(rrte_ctx* c) {
    rrte_ctx::Batch& b = c->batch;
    if (b.n == 0) return RRTE_OK;
    if (c->comm_failed || !c->comm) {
        b.n = b.nsrc = b.rendered = 0;
        return fail(c, RRTE_RCCL_ERROR, "gather batch dropped: %s", c->comm_failed ? c->comm_fail_msg.c_str() : "no communicator");
    }
    const bool launched_per_frame = b.per_frame;
    rrte_status r = launched_per_frame ? RRTE_OK : render_batch(c, true);
    if (r != RRTE_OK) return comm_abort(c, ("batch render failed: " + c->err).c_str());
    HostSection hs(c);
    const int k = c->bslot;
    const size_t count = (size_t)b.n * b.slice;  // bytes per rank
    auto issue = [&]() -> rrte_status {
        if (launched_per_frame) {
            // the frames rendered on their callers' streams: the exchange follows each of them
            for (uint32_t i = 0; i < b.nsrc; ++i) {
                HIPCHK(c, ev_record(c, b.ev_src[i], b.src[i], "record src (exchange)"));
                HIPCHK(c, ev_wait(c, c->comm_stream, b.ev_src[i], "comm waits src"));
            }
        } else {
            HIPCHK(c, ev_wait(c, c->comm_stream, c->ev_render[k], "comm waits render"));
        }
        if (c->last_gather_stream && c->last_gather_stream != c->comm_stream)
            HIPCHK(c, ev_wait(c, c->comm_stream, c->last_gather_ev, "comm waits last gather"));
        hs.lap(4);
        if ((r = before_collective(c, c->comm_stream)) != RRTE_OK) return r;
        // every peer's slab to the root: grouped point-to-point (the root's own bands never move); with
        // a 1-rank communicator (emulated ranks, RRTE_EMULATE_RANK) there is no peer, RRTE_GATHER_SELF
        // routes the root's bands through RCCL to itself
        const bool self_only = c->comm_size == 1;  // (no real peer: only the root's RRTE_GATHER_SELF round trip)
        if (!(c->env_diag_skip & 1u) && (!self_only || (!b.in_place && c->rank == b.root))) {
            // (a failing call inside the group still closes it before the error is returned, so the
            // thread's group depth is balanced when comm_abort tears the communicator down)
            NCCLCHK(c, ncclGroupStart());
            ncclResult_t gr = ncclSuccess;
            const char* what = "ncclRecv";
            if (c->rank == b.root) {
                for (int q = 0; q < c->comm_size && (gr == ncclSuccess || gr == ncclInProgress); ++q)
                    if (q != b.root || !b.in_place)
                        gr = ncclRecv(c->d_brecv[k] + (size_t)q * count, count, ncclUint8, q, c->comm, c->comm_stream);
            }
            if ((gr == ncclSuccess || gr == ncclInProgress) && (c->rank != b.root || !b.in_place)) {
                what = "ncclSend";
                gr = ncclSend(c->d_bsend[k], count, ncclUint8, b.root, c->comm, c->comm_stream);
            }
            const ncclResult_t er = ncclGroupEnd();
            if (gr != ncclSuccess && gr != ncclInProgress)
                return fail(c, RRTE_RCCL_ERROR, "%s failed: %s", what, ncclGetErrorString(gr));
            NCCLCHK(c, er);
        }
        if (self_only && c->emu_peers > 1 && c->rank == b.root &&
            (r = render_peers(c, b.plan, b.cam, b.n, c->d_brecv[k], count, b.slice, b.root, c->comm_stream)) != RRTE_OK)
            return r;
        hs.lap(5);
        if (c->rank == b.root && !(c->env_diag_skip & 2u) && (c->nranks > 1 || !b.in_place)) {
            DeinterleaveTargets t{};
            for (uint32_t j = 0; j < b.n; ++j) t.full[j] = b.full[j];
            if ((r = deinterleave(c, c->comm_stream, c->d_brecv[k], t, b.n, b.width, b.height, b.bm, b.rgb24, count,
                                  b.slice, b.in_place ? (uint32_t)b.root : ~0u)) != RRTE_OK)
                return r;
        }
        hs.lap(6);
        HIPCHK(c, ev_record(c, c->ev_batch[k], c->comm_stream, "record exchange done"));
        return RRTE_OK;
    };
    if ((r = issue()) != RRTE_OK) return comm_abort(c, ("batch gather failed: " + c->err).c_str());
    c->last_gather_stream = c->comm_stream;
    c->last_gather_ev = c->ev_batch[k];
    c->bslot = (k + 1) % c->batch_slabs;
    b.n = b.nsrc = b.rendered = 0;
    hs.lap(7);
    return RRTE_OK;
}

// One multi-GPU frame on `st`: render this rank's bands into its slice of a gather slab, gather it to
// the root and de-interleave there -- per frame (gather batch 1: everything on `st`, in place, the
// frames' gathers chained across streams in issue order), or batched (the gather happens when the
// open batch is full or flushed, on the comm stream).  `timing` (the blocking entry point): ev1 marks
// the end of the render for rrte_stats.
static rrte_status gather_frame(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, int root,
                                void* d_full, hipStream_t st, bool timing) {
    HostSection hs(c);
    rrte_status r = validate(c, s, p);
    if (r != RRTE_OK) return r;
    if (root < 0 || root >= c->nranks) return fail(c, RRTE_INVALID_ARG, "root %d out of range", root);
    if (c->rank == root && !d_full) return fail(c, RRTE_INVALID_ARG, "root needs an output buffer");
    double up = 0.0;
    hs.lap(0);
    if ((r = upload_scene(c, s, st, &up)) != RRTE_OK) return r;
    hs.lap(1);
    const uint32_t band = p->band_rows ? p->band_rows : 16;
    rrte_render_params pp = *p;
    pp.band_rows = band;
    uint32_t rows = p->height, cap = p->height;  // this rank's rows; slab rows (the most any rank owns)
    const bool rgb24 = slab_rgb24(c, s, p);
    // A frame joining an open batch of the same frame geometry keeps the batch's band partition: which
    // rank renders a band is a work-balance choice, never a pixel, and every rank makes the same one
    // from the same calls -- so a moving camera neither recomputes the partition every frame nor
    // closes the batch whenever its sky-band count changes
    const rrte_ctx::Batch& ob = c->batch;
    const bool join = c->nranks > 1 && c->gather_batch > 1 && !timing && ob.n && ob.width == p->width &&
                      ob.height == p->height && ob.band == band && ob.root == root && ob.rgb24 == rgb24;
    BandMap bm{band, 1u, 0u, 1u, 1u};
    if (join) {
        bm = ob.bm;
        rows = ob.plan.k.rows;
    } else if (c->nranks > 1) {
        bm = frame_band_map(c, s, &pp, root, &rows, &cap);
    }
    // bytes per rank slot, 256-B aligned so every rank's send buffer starts aligned
    const size_t slice = join ? ob.slice : ((size_t)cap * p->width * (rgb24 ? 3u : 4u) + 255u) & ~(size_t)255u;
    const uint32_t kflags = rgb24 ? kFlagSlabRgb24 : 0u;
    if (c->comm_failed)
        return fail(c, RRTE_RCCL_ERROR, "communicator aborted earlier (%s); call rrte_hip_comm_init", c->comm_fail_msg.c_str());
    // one rank: no exchange (RRTE_FORCE_GATHER=1 still takes the gather path: tests on one GPU)
    if (c->nranks == 1 && !(c->env_force_gather && c->comm)) {
        r = launch(c, s, p, p->height, static_cast<uint32_t*>(d_full), nullptr, st);
        if (r == RRTE_OK) c->pending_primary = (uint64_t)p->width * p->height * p->samples_per_pixel;
        if (timing) HIPCHK(c, hipEventRecord(c->ev1, st));
        return r;
    }
    if (!c->comm) return fail(c, RRTE_INVALID_ARG, "rrte_hip_comm_init has not been called");
    if (c->gather_batch > 1 && !timing) {
        rrte_ctx::Batch& b = c->batch;
        if (!c->comm_stream) {
            // the comm stream's gathers and de-interleaves at the highest priority: its kernels are
            // dispatched ahead of the next batches' render workgroups instead of queueing behind them
            // (RRTE_COMM_PRIORITY=0: default priority, A/B)
            int lo = 0, hi = 0;
            HIPCHK(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
            HIPCHK(c, hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, c->env_comm_priority ? hi : lo));
            for (int i = 0; i < c->batch_slabs; ++i) {  // (only the slots of the ring in use)
                HIPCHK(c, hipStreamCreateWithFlags(&c->render_stream[i], hipStreamNonBlocking));
                HIPCHK(c, hipEventCreateWithFlags(&c->ev_batch[i], hipEventDisableTiming));
                HIPCHK(c, hipEventCreateWithFlags(&c->ev_render[i], hipEventDisableTiming));
            }
            // one empty kernel on each new stream now: the runtime binds a stream to a hardware queue at
            // its first dispatch, which must not happen inside a later frame's critical path
            for (int i = 0; i < c->batch_slabs; ++i) {
                hipLaunchKernelGGL(noop_kernel, dim3(1), dim3(64), 0, c->render_stream[i]);
                HIPCHK(c, hipGetLastError());
            }
            hipLaunchKernelGGL(noop_kernel, dim3(1), dim3(64), 0, c->comm_stream);
            HIPCHK(c, hipGetLastError());
            for (int i = 0; i < rrte_ctx::kMaxBatch; ++i)
                HIPCHK(c, hipEventCreateWithFlags(&b.ev_src[i], hipEventDisableTiming));
        }
        LaunchPlan L = plan_launch(c, s, &pp, rows, kflags, 0u, &bm);
        // a frame of another size, band, root, slab format or render setup closes the open batch
        // (the cameras and tile rectangles are per frame; everything before KParams::nframes is not)
        if (b.n && (b.width != p->width || b.height != p->height || b.band != band || b.root != root ||
                    b.rgb24 != rgb24 || b.slice != slice || b.plan.mode != L.mode || b.plan.cull != L.cull ||
                    b.plan.single != L.single || memcmp(&b.plan.k, &L.k, offsetof(KParams, nframes))))
            if ((r = flush_batch(c)) != RRTE_OK) return r;
        const int k = c->bslot;
        if (b.n == 0) {
            b.cap = c->gather_batch;
            b.width = p->width;
            b.height = p->height;
            b.band = band;
            b.root = root;
            b.rgb24 = rgb24;
            b.slice = slice;
            b.bm = bm;
            b.plan = L;
            b.in_place = c->rank == root && !c->env_gather_self;
            b.per_frame = !c->env_batch_launch;
            // every rank holds a receive slab too (the root's is the only one written)
            const size_t send = (size_t)b.cap * slice, recv = send * (size_t)c->nranks;
            if (c->cap_bsend[k] < send || c->cap_brecv[k] < recv) {
                // every slab of the ring in use at once (at the first batch: none is allocated inside a
                // later timed batch); a smaller slab an in-flight gather may still use goes to the
                // graveyard (freed when the context is next idle), so nothing waits for the device here
                for (int q = 0; q < c->batch_slabs; ++q) {
                    if ((r = ensure(c, c->d_bsend[q], c->cap_bsend[q], send)) != RRTE_OK) return r;
                    if ((r = ensure(c, c->d_brecv[q], c->cap_brecv[q], recv)) != RRTE_OK) return r;
                }
            }
        }
        hs.lap(2);
        b.cam[b.n] = L.k.cam[0];
        b.cam[b.n].out = static_cast<uint32_t*>(d_full);
        b.full[b.n] = static_cast<uint32_t*>(d_full);
        uint32_t i = 0;
        while (i < b.nsrc && b.src[i] != st) ++i;
        const bool new_src = i == b.nsrc;
        if (new_src) b.src[b.nsrc++] = st;
        if (b.per_frame) {
            // render now, on the caller's stream: the root straight into the frame at its image rows
            // (RGBA8), a peer into its slot of the send slab -- after that slab's previous exchange
            // (once per stream and batch)
            if (b.in_place) {
                L.k.flags &= ~kFlagSlabRgb24;
                L.k.out_image_rows = 1u;
                L.k.cam[0].out = static_cast<uint32_t*>(d_full);
                if ((r = issue_launch(c, L, nullptr, nullptr, st)) != RRTE_OK) return r;
            } else {
                if (new_src) HIPCHK(c, hipStreamWaitEvent(st, c->ev_batch[k], 0));
                uint8_t* dst = c->d_bsend[k] + (size_t)b.n * b.slice;
                if ((r = issue_launch(c, L, reinterpret_cast<uint32_t*>(dst), nullptr, st)) != RRTE_OK) return r;
            }
            b.rendered = b.n + 1;
        }
        ++b.n;
        hs.lap(3);
        if (b.n == b.cap && (r = flush_batch(c)) != RRTE_OK) return r;
    } else {
        if ((r = flush_batch(c)) != RRTE_OK) return r;  // keep every rank's collectives in issue order
        if (!c->ev_gath[0])
            for (int i = 0; i < rrte_ctx::kSlabs; ++i)
                HIPCHK(c, hipEventCreateWithFlags(&c->ev_gath[i], hipEventDisableTiming));
        // slabs are a ring shared by every frame in flight: a frame on another stream than the slab's
        // previous user waits until that frame has been gathered (same stream: stream order suffices)
        const int slot = (int)(c->gather_frames % rrte_ctx::kSlabs);
        const size_t slab_words = slice * (size_t)c->nranks / 4u;
        if (c->cap_slab[slot] < slab_words) {
            // (re)size the whole ring at once; smaller slabs in-flight gathers may still use go to the
            // graveyard (freed when the context is next idle): no device synchronisation
            for (int i = 0; i < rrte_ctx::kSlabs; ++i)
                if ((r = ensure(c, c->d_slab[i], c->cap_slab[i], slab_words)) != RRTE_OK) return r;
        }
        uint8_t* slab = reinterpret_cast<uint8_t*>(c->d_slab[slot]);
        uint8_t* mine = slab + (size_t)c->rank * slice;  // in-place send slot
        if (c->slab_stream[slot] && c->slab_stream[slot] != st)
            HIPCHK(c, hipStreamWaitEvent(st, c->ev_gath[slot], 0));
        hs.lap(2);
        if ((r = launch(c, s, &pp, rows, reinterpret_cast<uint32_t*>(mine), nullptr, st, kflags, 0u, 0, &bm)) != RRTE_OK)
            return r;
        if (c->comm_size == 1 && c->emu_peers > 1 && c->rank == root) {  // RRTE_EMULATE_PEERS (tests)
            const LaunchPlan L = plan_launch(c, s, &pp, rows, kflags, 0u, &bm);
            if ((r = render_peers(c, L, L.k.cam, 1, slab, slice, 0, root, st)) != RRTE_OK) return r;
        }
        hs.lap(3);
        if (timing) HIPCHK(c, hipEventRecord(c->ev1, st));
        // gathers on one communicator must run in the same order on every rank: a frame on another
        // stream than the previous gather waits for it
        if (c->last_gather_stream && c->last_gather_stream != st)
            HIPCHK(c, hipStreamWaitEvent(st, c->last_gather_ev, 0));
        hs.lap(4);
        if ((r = before_collective(c, st)) != RRTE_OK) return comm_abort(c, ("gather setup failed: " + c->err).c_str());
        {
            const ncclResult_t nr = ncclGather(mine, slab, slice, ncclUint8, root, c->comm, st);
            if (nr != ncclSuccess && nccl_settle(c, nr, "ncclGather") != RRTE_OK) return comm_abort(c, c->err.c_str());
        }
        hs.lap(5);
        if (c->rank == root) {
            DeinterleaveTargets t{};
            t.full[0] = static_cast<uint32_t*>(d_full);
            if ((r = deinterleave(c, st, slab, t, 1, p->width, p->height, bm, rgb24, slice, 0)) != RRTE_OK)
                return comm_abort(c, ("de-interleave failed: " + c->err).c_str());
        }
        hs.lap(6);
        HIPCHK(c, hipEventRecord(c->ev_gath[slot], st));
        c->slab_stream[slot] = st;
        c->last_gather_stream = st;
        c->last_gather_ev = c->ev_gath[slot];
        hs.lap(7);
        ++c->gather_frames;
    }
    ++c->hp_frames;
    c->pending_primary = (uint64_t)p->width * rows * p->samples_per_pixel;
    c->stats.upload_ms = up;
    c->stats.frames++;
    return RRTE_OK;
}

rrte_status rrte_hip_render_gather_async(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, int root,
                                         void* d_full, void* stream) {
    if (!c) return RRTE_INVALID_ARG;
    dump_if_asked(c, s, p);
    return gather_frame(c, s, p, root, d_full, stream ? static_cast<hipStream_t>(stream) : c->stream, false);
}

rrte_status rrte_hip_set_gather_batch(rrte_ctx* c, uint32_t frames) {
    if (!c) return RRTE_INVALID_ARG;
    if (frames < 1 || frames > (uint32_t)rrte_ctx::kMaxBatch)
        return fail(c, RRTE_INVALID_ARG, "gather batch %u outside [1, %d]", frames, rrte_ctx::kMaxBatch);
    rrte_status r = flush_batch(c);
    if (r != RRTE_OK) return r;
    c->gather_batch = frames;
    return RRTE_OK;
}

rrte_status rrte_hip_flush(rrte_ctx* c) {
    if (!c) return RRTE_INVALID_ARG;
    return flush_batch(c);
}

rrte_status rrte_hip_host_register(rrte_ctx* c, void* host, size_t bytes) {
    if (!c || !host || bytes == 0) return fail(c, RRTE_INVALID_ARG, "null or empty host range");
    HIPCHK(c, hipSetDevice(c->device));
    unsigned flags = hipHostRegisterMapped;
    if (const char* g = getenv("RRTE_HOST_REGISTER_FLAGS")) flags = (unsigned)strtoul(g, nullptr, 0);  // (A/B)
    HIPCHK(c, hipHostRegister(host, bytes, flags));
    c->host_regs.push_back({host, bytes});
    return RRTE_OK;
}

rrte_status rrte_hip_host_unregister(rrte_ctx* c, void* host) {
    if (!c || !host) return RRTE_INVALID_ARG;
    for (size_t i = 0; i < c->host_regs.size(); ++i)
        if (c->host_regs[i].p == host) {
            HIPCHK(c, hipSetDevice(c->device));
            rrte_status r = rrte_hip_synchronize(c);  // (no frame may still write into it)
            if (r != RRTE_OK) return r;
            HIPCHK(c, hipHostUnregister(host));
            c->host_regs.erase(c->host_regs.begin() + (long)i);
            return RRTE_OK;
        }
    return fail(c, RRTE_INVALID_ARG, "host range %p was not registered with this context", host);
}

rrte_status rrte_hip_gather_info(rrte_ctx* c, uint64_t* collectives, uint32_t* open_frames) {
    if (!c || !collectives || !open_frames) return RRTE_INVALID_ARG;
    *collectives = c->gathers_issued;
    *open_frames = c->batch.n;
    return RRTE_OK;
}

rrte_status rrte_hip_render_gather(rrte_ctx* c, const rrte_scene_ir* s, const rrte_render_params* p, int root,
                                   uint8_t* out) {
    if (!c) return RRTE_INVALID_ARG;
    dump_if_asked(c, s, p);
    rrte_status r = validate(c, s, p);
    if (r != RRTE_OK) return r;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t npix = (size_t)p->width * p->height;
    uint32_t* full = nullptr;
    if (c->rank == root) {
        if ((r = ensure(c, c->d_full, c->cap_full, npix)) != RRTE_OK) return r;
        full = c->d_full;
    }
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    if ((r = gather_frame(c, s, p, root, full, c->stream, true)) != RRTE_OK) return r;
    HIPCHK(c, hipEventRecord(c->ev2, c->stream));
    if (c->rank == root && out) HIPCHK(c, hipMemcpyAsync(out, full, npix * 4, hipMemcpyDeviceToHost, c->stream));
    if ((r = wait_bounded(c)) != RRTE_OK) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float k_ms = 0.0f, all_ms = 0.0f;
    if (c->nranks > 1) {
        (void)hipEventElapsedTime(&k_ms, c->ev0, c->ev1);
        (void)hipEventElapsedTime(&all_ms, c->ev0, c->ev2);
        c->stats.kernel_ms = k_ms;
        c->stats.gather_ms = all_ms - k_ms;
    }
    return finish_frame(c);
}

}  // extern "C"
