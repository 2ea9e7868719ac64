/*
 * crt_scene_impl.h — the device scene behind the C-ABI handle (crt_hip_scene)
 * and the host layer's internal interface, shared by crt_host_render.hip
 * (plans, tables, launches, wavefront orchestration, shards) and crt_api.hip
 * (the extern "C" entry points of include/crt_hip.h).
 */
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "crt_bins.h"
#include "crt_host.h"
#include "crt_kernels.h"

#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        const hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                                    \
            return set_error(CRT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));      \
    } while (0)

namespace crt_amd {

struct ShardPlan {
    Tile *d_tiles = nullptr;
    int ntiles = 0;
    int waves = 0;               /* waves of the render grid (camera bins: the work lists' slots + rest tiles) */
    BinsPlan bp{};               /* camera-bins dispatch (crt_bins.hip bins_plan); cell_tile null otherwise */
    int64_t packed_pixels = 0;
    std::vector<Tile> tiles;     /* host copy, dispatch order */
    std::vector<float> cost;     /* measured cost per tile (calibrated plans), else empty */
    bool has_small = false;      /* some tile has <= 16 pixels (walk 13 runs them with the window walk) */
};

}  // namespace crt_amd

using namespace crt_amd;

/* Flags of the events that order the frames pipelines' streams on one device
 * (camera bins, wavefront sets): no timing, and no system-scope fence — the
 * work they order is on the same device, and kernel ends release to it. */
#ifndef CRT_PIPE_EV_FLAGS
#define CRT_PIPE_EV_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif

/* Device buffers of the camera bins (crt_bins.hip), per scene. */
struct BinsDev {
    crt_amd::BinCamera cam{};
    int nt = 0, tx = 0, ncell = 0;
    crt_amd::CamCand *tpl = nullptr;      /* per triangle: the records' static part */
    crt_amd::BinItem *items = nullptr;    /* per triangle: this frame's projection */
    int32_t *tpref = nullptr;             /* per triangle: pair prefix inside its group of k_bins_project */
    int32_t *gsum = nullptr;              /* per group: pairs */
    int32_t *rem = nullptr;               /* groups queued for k_bins_pairs */
    int pair_blocks = 0;                  /* k_bins_pairs grid (0: not launched; the sizing pass queued none) */
    int qmax = 8192;                      /* groups k_bins_pairs takes (kMaxGroups; option "bins_qmax" lowers it) */
    int32_t *cnt = nullptr;               /* per cell: candidates; kBinSets sets (a frame zeroes the next one's) */
    uint64_t *keys = nullptr;             /* per cell: kBinCellCap sort keys (dmin bits << 32 | triangle id) */
    int32_t *every = nullptr;             /* everywhere triangles */
    int32_t *nonempty = nullptr;          /* cells with a candidate: kBinShards lists of cap_shard, arrival order */
    int32_t *bigl = nullptr;              /* cells of more than 16 candidates: kBinShards lists of cap_shard */
    int cap_shard = 0;
    int long_waves = 0;                   /* k_bins_sort waves for the long lists */
    crt_amd::BinsHdr *hdr = nullptr;      /* kBinSets sets: frames take them in turn */
    uint64_t frame = 0;                   /* frames binned (set = frame % kBinSets) */
    /* the last binning: its set, camera and plan (the work lists it wrote).
     * A frame with the same camera and plan renders that set again instead of
     * binning (the lists are a function of the camera: option "bins_reuse") */
    int last = -1;
    crt_amd::BinCamera binned{};
    const void *binned_plan = nullptr;
    int64_t binnings = 0, reuses = 0;
    crt_amd::BinsCaps caps{};             /* per shard: its region of recs */
    crt_amd::CamCand *recs = nullptr;     /* the lists, kBinSets sets (rec_cap each) */
    int32_t rec_cap = 0;
    int32_t *off = nullptr, *len = nullptr;   /* per cell, kBinSets sets (ncell each) */
    std::vector<int32_t> count;           /* per cell: list length of the sizing pass (-1 over the cap) */
    int sort_blocks = 0;                  /* k_bins_sort blocks */
    int64_t records = 0;                  /* records of the sizing pass */
    double setup_ms = 0.0;
    std::vector<void *> allocs;           /* the view's buffers (bins_free_view) */
    std::vector<void *> keep;             /* per triangle: templates, items and the projection's scratch */
    /* frames pipeline: frame k's binning runs on `stream` (its kernels in
     * order) while frame k - 1 renders; the lists the render reads come in
     * kBinSets sets taken in turn, bdone[p] = set p's lists built, rdone[p] =
     * set p's render done with them */
    hipStream_t stream = nullptr;
    hipEvent_t bdone[crt_amd::kBinSets] = {}, rdone[crt_amd::kBinSets] = {};
    hipStream_t bdone_s[crt_amd::kBinSets] = {}, rdone_s[crt_amd::kBinSets] = {};   /* where each was last recorded */
};


/* One frame's buffers of the wavefront path, grown on demand (kept across
 * frames).  Up to kWfSets sets: recorded-size frames take them in turn, set
 * i's levels on stream i % kWfStreams, so the levels of several consecutive
 * frames run side by side (render_wavefront); frames with read-backs use set
 * 0 on the caller's stream. */
struct WfSet {
    crt_amd::WNode *nodes = nullptr;
    crt_amd::DVec4 *cols = nullptr;
    int64_t cap = 0;             /* ray ids */
    crt_amd::WRay *q[2] = {nullptr, nullptr};
    int64_t qcap[2] = {0, 0};
    int32_t *counts = nullptr;   /* children queued per level; counts[count_cap - 1]: overflow flag */
    int count_cap = 0;
    /* overflow flag of recorded-size frames: device word, copied into pinned
     * host memory behind each such frame and read once that copy is done */
    int32_t *d_flag = nullptr;
    int32_t *h_flag = nullptr;
    hipEvent_t flag_ev = nullptr;
    bool flag_pending = false;
    hipEvent_t free_ev = nullptr;     /* the set's last frame has written its pixels */
    uint64_t seq = 0;                 /* WfBuffers::frame of the set's last frame */
    hipEvent_t done_ev = nullptr;     /* the set's levels of the current frame are done */
    /* a device-sized frame's level sizes, copied back behind it to record them
     * (WfBuffers::Rec) once they land, if the camera has not moved since */
    int32_t *h_counts = nullptr;      /* pinned, kWfDynMaxLevels */
    hipEvent_t counts_ev = nullptr;
    bool counts_pending = false;
    const void *counts_tiles = nullptr;
    crt_renderer_settings counts_st{};
    int counts_ntiles = 0;
    int counts_levels = 0;
    int64_t counts_qcap = 0;
    int64_t counts_idcap = 0;         /* ray ids the frame's levels could take */
    uint32_t rec_slots = 0;           /* device record ring slots the set's frames read (their levels, on the set's
                                       * stream) since that slot was last reused */
    uint64_t counts_epoch = 0;
};

#ifndef CRT_WF_SETS
#define CRT_WF_SETS 12           /* wavefront frame buffer sets, at most (A/B builds: 2, 4, 8, 16) */
#endif
#ifndef CRT_WF_STREAMS
#define CRT_WF_STREAMS CRT_WF_SETS
#endif
#ifndef CRT_WF_SET_BUDGET
#define CRT_WF_SET_BUDGET (16ll << 30)   /* bytes all sets of one frame size may take together */
#endif
constexpr int kWfSets = CRT_WF_SETS;
constexpr int kWfStreams = CRT_WF_STREAMS;    /* set i's levels run on stream i % kWfStreams */
static_assert(kWfSets % kWfStreams == 0, "buffer sets share streams evenly");
static_assert(kWfSets >= 2, "frames in flight need two sets at least");
struct WfBuffers {
    WfSet set[kWfSets];
    hipStream_t streams[kWfStreams] = {};
    uint64_t frame = 0;          /* recorded-size frames issued */
    /* Level sizes of the last frame traced with host read-backs, and what they
     * depend on (settings, tile list): a frame's level sizes are a function of
     * its rays alone, so later frames with the same key launch every level
     * with these sizes and no host sync (render_wavefront). */
    struct Rec {
        std::vector<int32_t> sizes;   /* rays of levels 1, 2, ... */
        crt_renderer_settings st{};
        int ntiles = 0;
    };
    std::map<const void *, Rec> recs;   /* by tile list (device pointer; cleared when plans are freed) */
    bool force_readback = false;        /* after an overflow: the next frame reads its sizes back */
    bool shrink_records = false;        /* option wf_replay 2 (tests): sizes recorded minus one */
    uint64_t epoch = 0;                 /* bumped whenever recs are dropped (a device-sized frame's sizes
                                         * are recorded only if no drop happened since it was issued) */
    /* recorded-size frames captured as HIP graphs, by everything their
     * launches bake in (cleared whenever a buffer, tile list or record changes) */
    struct Graph {
        const void *tiles;
        crt_renderer_settings st;
        const float *out;
        hipStream_t stream;
        int set;                 /* the buffer set whose pointers the graph holds */
        const void *scene;
        hipGraphExec_t exec;
    };
    std::vector<Graph> graphs;
};

/* Device scene records in flight (crt_host_render.hip sync_device_record). */
constexpr int kRecRing = 16;
static_assert(kRecRing <= 32, "WfSet::rec_slots is a 32-bit mask of ring slots");

/* Deepest recursion the wavefront path accepts (levels are launched one by one). */
constexpr int kWfMaxDepth = 4096;
/* device-sized wavefront frames (render_wavefront): up to this max_ray_depth + 2 levels */
constexpr int kWfDynMaxLevels = 66;

struct crt_hip_scene {
    int device = 0;
    /* Multi-GPU behind one handle (crt_multi.hip): further replicas of the
     * scene (this one is replica 0), the gather buffer on this device and, on
     * a replica, its packed shard and the event that its copy is done. */
    std::vector<crt_hip_scene *> replicas;
    float *mg_gather = nullptr;
    int64_t mg_gather_floats = 0;
    float *mg_packed = nullptr;
    int64_t mg_packed_floats = 0;
    hipEvent_t mg_done = nullptr;     /* replica: its shard is copied | replica 0: the gather is unpacked */
    crt_scene_info info{};
    bool has_secondary = false;    /* any reflective / refractive material */
    bool has_diffuse = false;
    bool has_refractive = false;   /* Fresnel term: needs the powf table (fresnel_of) */
    DeviceScene ds{};
    DeviceScene ds_uploaded{};   /* what d_ds holds */
    DeviceScene *d_ds = nullptr;     /* the current record: a slot of d_ring (sync_device_record) */
    DeviceScene *d_ring = nullptr;
    int ring_cur = -1;
    hipStream_t rec_up_stream = nullptr;   /* where the current record was written */
    bool rec_up_done = false;              /* ... and the write is done */
    bool rec_up_recorded = false;          /* rec_up of the current slot recorded (a reader on another stream) */
    hipStream_t rec_last_stream = nullptr;  /* where the last frame that read the current record was issued */
    bool rec_read_by_set = false;          /* the frame just issued read it on a wavefront set's stream
                                            * (WfSet::rec_slots + done_ev cover it, not rec_last_stream) */
    hipEvent_t rec_up[kRecRing] = {};    /* slot written */
    hipEvent_t rec_use[kRecRing] = {};   /* the last frame that read the slot is done */
    hipStream_t rec_use_stream[kRecRing] = {};   /* where each slot's last frame was issued (null: none) */
    int64_t records_written = 0;
    crt_wave_counts wave_counts{};   /* from the last crt_hip_count_work */
    std::vector<void *> allocs;
    hipStream_t stream = nullptr;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    /* crt_hip_render into pageable host memory (stage_to_host): a pinned
     * staging image and one event per chunk of the copy */
    float *h_stage = nullptr;
    std::vector<hipEvent_t> stage_ev;
    /* the compact image copy (crt_api.hip image_to_host): per row of the
     * frame its span of non-background pixels, on the device and in pinned
     * memory (k_row_spans), and the ends of the two copy kernels */
    crt_amd::HostRow *h_rows = nullptr;
    int2 *d_row_spans = nullptr;
    int32_t copy_h = 0;
    hipEvent_t spans_ev = nullptr, copy_ev = nullptr;
    hipEvent_t copy_band_ev[4] = {};   /* staged copies: the end of each band of rows' launch */
    int compact_copy = 1;          /* option "compact_copy": 0 copies the whole image */
    ShardPlan full;
    std::map<std::pair<int, int>, ShardPlan> shard_plans;
    std::map<int, std::pair<UnpackBucket *, int>> unpack_plans;
    /* compact shards (crt_hip_*_compact): live-pixel mask of the frame (host),
     * per-(shard, count) render plans, per-count unpack lists */
    std::vector<uint8_t> live_mask;
    std::map<std::pair<int, int>, ShardPlan> compact_plans;
    std::map<int, std::pair<UnpackBucket *, int>> compact_unpack;
    float *d_out = nullptr;
    unsigned long long *d_counters = nullptr;
    int32_t *d_next_px = nullptr;      /* pixel-refill list head (k_render_refill) */
    int gi_refill = 1;                 /* GI frames: persistent waves with pixel refill (env CRT_GI_REFILL, option "gi_refill") */
    int gi_machine = 1;                /* ... as per-lane state machines (k_render_gi; option "gi_machine") */
    int rec_machine = 0;               /* recursion without GI through the same state machine (option "rec_machine") */
    int gi_blocks = 1024;              /* blocks of the k_render_gi grid (resident blocks per CU x CUs) */
    /* deferred shadow rays (option "shadow_defer", crt_host_render.hip
     * launch_shadow_frame): records of the frame's groups, its counter */
    int shadow_defer = 1;   /* (C2 with shadows: 0.396 ms deferred with light bins, 0.416 inline BVH walks, 0.427 inline light bins) */
    void *sh_buf = nullptr;
    int64_t sh_bytes = 0;
    int32_t *sh_count = nullptr;
    hipEvent_t sh_done = nullptr;      /* after the last deferred frame's compose */
    hipStream_t sh_stream = nullptr;   /* ... on this stream */
    void *gi_frames = nullptr;         /* k_render_gi: frames below the LDS ones (grown on demand) */
    int64_t gi_frames_bytes = 0;
    int refill_waves = 5120;           /* waves of the refill grid: CUs x 4 SIMDs x CRT_GI_WAVES */
    bool grid_empty = false;
    int traversal = 8;             /* 7 reference order | 8 pruned (default), see trace<> (env CRT_TRAVERSAL) */
    int shadows = 0;               /* option "shadows": trace the shadow rays (k_render_tiles<..., SHADOW>) */
    int light_bins = 1;            /* option "light_bins": shadow rays over the light bins (ensure_light_bins) */
    bool lbins_tried = false;      /* built (or found not to apply) at the first shadow-ray frame */
    int lbins_n = 0;               /* their cells a cube-face side (0: none) */
    int64_t lbins_records = 0;
    double lbins_ms = 0.0;
    int trace_walk = 1;            /* crt_hip_trace_batch: 0 reference-order walk, 1 pruned per-lane walk */
    float fov_radians = 0.f;       /* the camera's (ds.cam: the rest) */
    int64_t camera_moves = 0;      /* crt_hip_scene_set_camera calls that changed the camera */
    int64_t view_rebuilds = 0;     /* ... of them that rebuilt plans and buffers with the device drained */
    float prune_origin_max = 0.f;  /* the hull margins' origin bound (bins need the camera inside it) */
    bool camera_fast = false;      /* every camera ray takes the fast box path (camera_rays_fast) */
    /* estimate plan (no calibration): a tile is split into 4x4 (2x2) pixel
     * waves when its work estimate exceeds split4 (split16) times the mean work
     * per resident wave slot, i.e. when it would run for several times the
     * ideal makespan */
    float split4 = 4.5f, split16 = 9.0f;
    int wave_slots = 6144;   /* CUs x 4 SIMDs x 6 resident render waves */
    int secondary = 0;       /* walk for secondary rays: 0 = by frame, 4, 10 (env CRT_SECONDARY) */
    std::vector<float> tile_work;  /* per 8x8 tile of the full frame */
    BinsDev bins;                  /* camera bins (crt_bins.hip) */
    /* measured-cost tile plan (calibrate_plan): per 8x8 tile of the full frame,
     * the sub-tiles it is split into and their probed costs */
    struct SubTile { int32_t dx, dy, w, h; float cost; };
    std::vector<std::vector<SubTile>> calib;
    int calib_walk = -1;           /* primary walk the calibration was measured with (-1: none) */
    int calibrate = 2;             /* 0 estimate plan, 1 measured costs with a tuned k (10 candidate plans, 6 frames
                                    * each, on the first frame: long-running hosts, bench.py), 2 (default: one-shot
                                    * callers pay one calibration, no tuning frames) measured costs with calib_k */
    int window_walk = 1;           /* camera walk 12 -> 13 (window walk for split tiles), env CRT_WINDOW */
    int record_events = 1;         /* start/stop events around every render (crt_hip_last_kernel_ms), option "events" */
    bool events_valid = false;
    float calib_k = 2.25f;         /* split a wave whose cost exceeds k x (total cost / wave slots); 2.25 = C2's
                                    * tuned k (profiles/r02/gab, shard_kscan) */
    int calib_min = 2;             /* smallest sub-tile side */
    bool calib_tuned = false;      /* calibrate 1: k was tuned (once per scene and resolution; a later walk — a
                                    * camera move between fast and slow poses — calibrates with it, no trial frames) */
    bool calib_defer = true;       /* calibrate 2 (one-shot default): a walk's first frame renders with the
                                    * current plan and the calibration runs on its second frame (off once the
                                    * caller sets calibrate / calib_k_milli / calib_min) */
    int calib_deferred_walk = -1;  /* walk whose first frame skipped the calibration */
    int bins_on = 1;               /* camera frames take the camera bins where built (walk 15; option "bins") */
    int64_t bins_mean_cap = crt_amd::kBinMeanCap;   /* candidates per cell on average, at most (env CRT_BINS_MEAN_CAP) */
    int wf_dynamic = 1;            /* wavefront frames without recorded sizes: device-sized levels, no read-back (option "wf_dynamic") */
    int wf_record = 1;             /* frames replay recorded level sizes (HIP graphs) when they have them; 0: every
                                    * frame device-sized (option "wf_record") */
    int wf_dyn_ids = 4;            /* ... their ray-id capacity, x camera rays (option "wf_dyn_ids") */
    int wf_dyn_waves = 8192;       /* ... the waves of each level's grid, at most (option "wf_dyn_waves") */
    int bvh_device = 1;            /* build the BVH on the device above kHostBvhMax triangles (create flag
                                    * CRT_SCENE_NO_DEVICE_BVH: not) */
    int create_flags = 0;          /* the create's CRT_SCENE_* flags (crt_multi.hip: the probe's test hook) */
    int bins_slack = 100;          /* camera-bins grid slots per kind: the sizing pass's count + this % (option "bins_slack") */
    int bins_reuse = 1;            /* a frame whose camera the last binning used renders its lists (option "bins_reuse") */
    int bins_split = 48;           /* cells with this many candidates run as four 4x4 waves (option "bins_split") */
    int bins_quad = 1;             /* those waves walk with four lanes per pixel (option "bins_quad") */
    void *probe_buf = nullptr;     /* calibration probes: tile list + costs (probe_tiles) */
    size_t probe_cap = 0;          /* bytes */
    int prio_tiles = 1024;         /* heaviest tiles run at raised issue priority */
    float prio_min = 2.0f;         /* ... if they cost more than this x the mean per wave slot */
    std::vector<void *> plan_allocs;   /* tile lists of the current plans */
    /* the tree in the reference's numbering (crt_hip_scene_tree): host copies
     * for a host-built tree, device arrays for a device-built one */
    std::vector<float> ref_bounds;
    std::vector<int32_t> ref_children, ref_leaf_tris;
    std::vector<int64_t> ref_leaf_off;
    const float *dt_ref_bounds = nullptr;
    const int32_t *dt_ref_children = nullptr, *dt_ref_leaf_tris = nullptr;
    const int64_t *dt_ref_leaf_off = nullptr;
    int wavefront = 1;             /* level-by-level recursion when GI is off (env CRT_WAVEFRONT) */
    int wf_graph = 1;              /* recorded-size wavefront frames replayed from captured HIP graphs (option "wf_graph") */
    int wf_replay = 1;             /* wavefront frames after the first: 1 recorded level sizes, 0 read back every level,
                                    * 2 recorded sizes minus one (tests: forces the overflow path) (option "wf_replay") */
    int wf_rays_per_wave = 48;     /* cap on the rays per wave of wavefront levels >= 1 (each level takes
                                    * min(cap, max(8, n / 4096)), render_wavefront), coop walks (env CRT_WF_RPW,
                                    * option "wf_rpw"); fixed 48 / 32 / 16 / 64: 3.55 / 3.64 / 3.62 / 3.68 ms */
    WfBuffers wf;
};

namespace crt_amd {

void wf_graphs_clear(WfBuffers &w);
void wf_free(WfBuffers &w);
bool wf_overflowed(WfBuffers &w, bool wait);
int wf_streams(WfBuffers &wb, hipStream_t stream);
int make_tile_plan(crt_hip_scene *sc, const std::vector<DBucket> &buckets, bool full_frame, ShardPlan &plan);
void free_plans(crt_hip_scene *sc);
int sync_device_record(crt_hip_scene *sc, const DeviceScene **out, hipStream_t stream);
int wait_device_record(crt_hip_scene *sc, hipStream_t stream);
int used_device_record(crt_hip_scene *sc, hipStream_t stream);
int check_settings(const crt_renderer_settings *st);
int ensure_plans(crt_hip_scene *sc, const crt_renderer_settings *st, hipStream_t stream, bool render = false);
void warm_code_objects(int device, hipStream_t stream);
void start_host_tables(bool gi, bool pow5);
int ensure_gi_tables(crt_hip_scene *sc);
int ensure_pow5_table(crt_hip_scene *sc);
int ensure_light_bins(crt_hip_scene *sc, const crt_renderer_settings *st);
/* camera frames of this scene walk the camera bins (walk 15): built, enabled,
 * and the default camera walk selected */
inline bool bins_active(const crt_hip_scene *sc) { return sc->ds.bins && sc->bins_on && sc->traversal == 14; }
int launch_render(crt_hip_scene *sc, const crt_renderer_settings *st, const ShardPlan &plan, float *d_out,
                  hipStream_t stream, bool count, unsigned long long *stamps = nullptr);
int render_into(crt_hip_scene *sc, const crt_renderer_settings *st, float *d_rgb, hipStream_t stream, bool count);
bool camera_rays_fast(const DCamera &c, bool planes_ok);
bool rec_machine_on(const crt_hip_scene *sc, const crt_renderer_settings *st);
int ensure_live_mask(crt_hip_scene *sc);
std::vector<DBucket> compact_tiles(crt_hip_scene *sc, int shard, int shard_count, int64_t *px,
                                   std::vector<DBucket> *dead = nullptr);
int render_shard_t(crt_hip_scene *sc, const crt_renderer_settings *st, int shard, int shard_count, float *d_packed,
                   void *stream, bool compact);
template <class T>
int unpack_shards_t(crt_hip_scene *sc, int shard_count, const T *d_gathered, T *d_rgb, void *stream, bool compact);
int scene_upload_buffers(crt_hip_scene *sc, const HostScene &hs);
int scene_upload(const HostScene &hs, int device, bool primary, crt_hip_scene **out);
/* crt_bins.hip: camera bins built on the device by every camera frame */
int bins_setup(crt_hip_scene *sc, const HostScene &hs);
int bins_view(crt_hip_scene *sc);
void bins_free_view(crt_hip_scene *sc);
int bins_plan(crt_hip_scene *sc, ShardPlan &plan);
int bins_enqueue(crt_hip_scene *sc, const ShardPlan &plan, hipStream_t s, int *par_out, bool force = false);
void bins_free(crt_hip_scene *sc);
/* crt_multi.hip: the frame over every replica of a multi-GPU scene into d_rgb
 * (on the scene's device) on `stream`; *overflow: some replica's recorded
 * wavefront sizes did not hold (render again). */
int render_multi_into(crt_hip_scene *sc, const crt_renderer_settings *st, float *d_rgb, hipStream_t stream);
bool multi_overflowed(crt_hip_scene *sc);
void multi_free(crt_hip_scene *sc);

/* The scene's arrays in one device allocation and one copy (scene_upload):
 * add() appends an array (copied at once: it may be a temporary) and records
 * where its device pointer goes; flush() allocates once, copies once and sets
 * the pointers.  A separate allocation and synchronous copy per array cost
 * ~0.3 ms each on a warm device. */
class UploadBatch {
public:
    template <class T>
    void add(const std::vector<T> &v, const T **dst, size_t pad = 0) {
        /* pad: zeroed records after the data, so grouped reads past a run's end stay in bounds */
        *dst = nullptr;
        if (v.empty() && pad == 0) return;
        const size_t off = host_.size(), n = v.size() * sizeof(T), all = n + pad * sizeof(T);
        host_.resize((off + all + 255) & ~size_t(255), 0);
        if (n) std::memcpy(host_.data() + off, v.data(), n);
        items_.push_back(Item{reinterpret_cast<const void **>(dst), off});
    }
    int flush(crt_hip_scene *sc);

private:
    struct Item {
        const void **dst;
        size_t off;
    };
    std::vector<Item> items_;
    std::vector<char> host_;
};

template <class T>
int upload(crt_hip_scene *sc, const std::vector<T> &v, const T **dst, size_t pad = 0) {
    /* pad: zeroed records after the data, so grouped reads past a run's end stay in bounds */
    *dst = nullptr;
    if (v.empty() && pad == 0) return CRT_OK;
    void *p = nullptr;
    const size_t bytes = (v.size() + pad) * sizeof(T);
    HIP_TRY(hipMalloc(&p, bytes));
    sc->allocs.push_back(p);
    if (pad) HIP_TRY(hipMemset(static_cast<char *>(p) + v.size() * sizeof(T), 0, pad * sizeof(T)));
    if (!v.empty()) HIP_TRY(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    sc->info.device_bytes += (int64_t)bytes;
    *dst = static_cast<const T *>(p);
    return CRT_OK;
}

}  // namespace crt_amd
