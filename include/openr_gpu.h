/*
 * openr_gpu.h — C-ABI of the MI355X (gfx950) SPF + RouteDb engine for Open/R
 * Decision. This is the drop-in boundary: plain pointers and sizes, int
 * status codes, no exceptions and no C++/torch types across the ABI.
 *
 * The reference has no FFI for this path; its C++ API is
 *   LinkState::getSpfResult   (openr/decision/LinkState.h:358-359,
 *                              LinkState.cpp:705-820)
 *   LinkState::getKthPaths    (LinkState.h:383-384, LinkState.cpp:674-703)
 *   SpfSolver::buildRouteDb   (openr/decision/SpfSolver.h:136-139,
 *                              SpfSolver.cpp:160-453)
 *   RibPolicy::applyPolicy    (openr/decision/RibPolicy.cpp:231-249)
 *   DecisionRouteDb::calculateUpdate (SpfSolver.cpp:21-56)
 * The C++ adapter in openr_amd/csrc/host keeps exactly those signatures and
 * calls the entry points below; INTEGRATION.md shows the binding.
 *
 * Data layout (all arrays DEVICE-resident unless stated):
 *   A "graph batch" holds T independent topologies in one CSR. Node ids are
 *   local to their topology and equal the rank of the node name in byte-wise
 *   sorted order, so id order == the reference's name tie-break order.
 *   Each directed edge is one uint64:
 *     bits  0..20  dst   local node id of the neighbour
 *     bit  21      DST_OVERLOADED  neighbour is hard-drained: it is settled
 *                  but never relaxes (LinkState.cpp:741-752) unless it is
 *                  the SPF source itself
 *     bits 22..30  rslot index of the reverse edge inside dst's CSR row,
 *                  saturated at 511 (rows of 512+ edges: ogs_graph.rslot_ext)
 *     bit  31      DOWN  link not up (Link::isUp false, LinkState.h:118-121)
 *     bits 32..63  metric (Link::getMaxMetric, LinkState.h:171-174)
 *   Node flags (uint8): OGS_NODE_OVERLOADED (hard drain, no transit,
 *   LinkState.cpp:741-752), OGS_NODE_SOFTDRAIN (int(metricInc) > 0,
 *   SpfSolver.cpp:518-519), OGS_NODE_METRICINC (metricInc != 0,
 *   SpfSolver.cpp:549-550).
 *   Next-hop sets are bitsets over the SOURCE node's CSR row ("link slots"):
 *   bit j of a node's set <=> the j-th link of the source is an ECMP first
 *   hop toward it (the union rule of LinkState.cpp:795-811 composed with the
 *   link filter of SpfSolver.cpp:705-743).
 */
#ifndef OPENR_GPU_H_
#define OPENR_GPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of this header: a consumer checks ogs_abi_version() ==
 * OGS_ABI_VERSION once at start-up. 3: ogs_spf_out.reached,
 * ogs_area_table.reached, ogs_routes_from_spf(spf_reached), u16 RibPolicy
 * statement ids, ogs_graph.rslot_ext (rows of 511+ edges). 4:
 * ogs_spf_routes_variants writes ogs_route_diff.base_desc_valid back. 5:
 * ogs_spf_routes_groups / ogs_route_group. 6: execution contexts
 * (ogs_ctx_create / ogs_ctx_set_option / ogs_ctx_* compute calls). */
#define OGS_ABI_VERSION 6

/* ---- status codes ------------------------------------------------------ */
#define OGS_OK 0
#define OGS_E_INVALID (-1)     /* bad argument / inconsistent shapes         */
#define OGS_E_NOMEM (-2)       /* device allocation failed                   */
#define OGS_E_HIP (-3)         /* HIP runtime error, see ogs_last_error()    */
#define OGS_E_UNSUPPORTED (-4) /* input the encodings cannot hold: > 2^21  */
                               /* nodes per topology, an OGS_F_EXACT_ORDER */
                               /* call without u64 distances               */
#define OGS_E_NODEVICE (-5)    /* no HIP device visible                      */

/* ---- packed edge / node encodings -------------------------------------- */
#define OGS_EDGE_DST_BITS 21
#define OGS_EDGE_DST_MASK 0x1FFFFFu
#define OGS_EDGE_DST_OVERLOADED (1u << 21)
#define OGS_EDGE_RSLOT_SHIFT 22
#define OGS_EDGE_RSLOT_MASK 0x1FFu
#define OGS_EDGE_DOWN (1u << 31)
#define OGS_MAX_NODES_PER_TOPO (1u << 21)
/* Rows up to this length fit the 9-bit reverse slot; longer rows need
 * ogs_graph.rslot_ext. Next-hop sets of sources past 512 links are wider than
 * 16 words (ogs_nh_words_for_degree). */
#define OGS_MAX_DEGREE 512

#define OGS_NODE_OVERLOADED 0x01u
#define OGS_NODE_SOFTDRAIN 0x02u
#define OGS_NODE_METRICINC 0x04u
#define OGS_NODE_NONE 0xFFFFFFFFu /* advertiser with no adjacency database */

#define OGS_PFX_V4 0x01u
#define OGS_PFX_HAS_MIN_NH 0x02u

/* ---- route record flags (ogs_route_out.meta) --------------------------- */
#define OGS_ROUTE_VALID 0x01u       /* a unicast route exists              */
#define OGS_ROUTE_DRAINED 0x02u     /* isBestNodeDrained -> drain_metric=1 */
#define OGS_ROUTE_LOCAL 0x04u       /* localRouteConsidered                */
#define OGS_ROUTE_SELECTED 0x08u    /* selection ran (bestRoutesCache set) */
#define OGS_ROUTE_REASON_SHIFT 4    /* 4-bit reason when not VALID         */
#define OGS_ROUTE_BEST_SHIFT 8      /* best advertiser index in segment    */
#define OGS_REASON_NONE 0
#define OGS_REASON_V4_DISABLED 1    /* SpfSolver.cpp:169-176 */
#define OGS_REASON_UNREACHABLE 2    /* SpfSolver.cpp:217-223 */
#define OGS_REASON_SELF 3           /* SpfSolver.cpp:253-258 */
#define OGS_REASON_NO_NEXTHOP 4     /* SpfSolver.cpp:605-607 */
#define OGS_REASON_MIN_NEXTHOP 5    /* SpfSolver.cpp:612-619 */

/* ---- solver flags ------------------------------------------------------- */
#define OGS_F_ENABLE_V4 0x01u          /* SpfSolver ctor enableV4          */
#define OGS_F_V4_OVER_V6 0x02u         /* v4OverV6Nexthop                  */
#define OGS_F_BEST_ROUTE_SELECTION 0x04u /* enableBestRouteSelection       */
#define OGS_F_HOP_METRIC 0x08u         /* getSpfResult(useLinkMetric=false)*/
#define OGS_F_WIDE_METRIC 0x10u        /* 64-bit distances (else 32-bit)   */
/* Settle nodes in the reference's DijkstraQ order (smallest (metric, node
 * name), LinkState.h:618-626) instead of solving the order-free fixpoint:
 * exact for zero link metrics and for negative i32 metrics (edge metric =
 * the sign-extended i32, u64 sums wrap, LinkState.cpp:77-78, 789). Needs
 * OGS_F_WIDE_METRIC; one wavefront per unit, one extraction per step. */
#define OGS_F_EXACT_ORDER 0x20u
/* ogs_spf_routes_variants only: repair the base unit's SPF (diff->base_dist /
 * base_nh) instead of recomputing it -- only nodes below a failed link that
 * was tight in the base shortest-path DAG are re-relaxed; next-hop sets of
 * one word (nh_words 1), else the full recompute runs. */
#define OGS_F_INCREMENTAL 0x40u
/* ogs_spf_routes_variants only (with a diff): write only the records of
 * changed routes (bit set in diff->changed); the other records of out->meta
 * / metric / mask / sel are left as they were. Needs OGS_F_INCREMENTAL. */
#define OGS_F_CHANGED_ONLY 0x80u

/* CSR of T topologies. */
typedef struct ogs_graph {
  int32_t num_topos;
  int32_t max_nodes;          /* max node count of any topology          */
  int32_t max_edges;          /* max directed-edge count of any topology */
  int32_t max_degree;         /* max CSR row length of any node          */
  const uint32_t* node_base;  /* [T+1] first global node of topology t   */
  const uint32_t* row_ptr;    /* [total_nodes+1] global edge offsets     */
  const uint64_t* edges;      /* [E] packed as above                     */
  const uint8_t* node_flags;  /* [total_nodes]                           */
  /* Optional [T*8] per-topology descriptor {node_base, nodes, edge_base,
   * edges, pfx_base, prefixes, adv_base, advertisements} (prefix fields 0
   * without a prefix table). Redundant with the arrays above; lets a unit
   * fetch all its offsets with one load instead of a dependent chain. */
  const uint32_t* topo_desc;
  /* Optional [T*slot_stride] relaxation order for the wave-per-unit path:
   * position i of topology t holds a node id (0xFFFF = empty); position i
   * is processed in slot i/64 by lane i%64. Any permutation is exact; the
   * adapter 2-colours the topology so consecutive slots alternate colour
   * classes and one round propagates two hops on bipartite graphs.
   * slot_stride is 64, 128 or 256 (0 with slot_node NULL). */
  const uint16_t* slot_node;
  int32_t slot_stride;
  /* Optional [T][slot_degree][slot_stride] per-position edge image for the
   * wave path (requires slot_node; all metrics <= 65535, degree <= 8):
   * entry j of position i is the i-th ordered node's j-th CSR edge,
   *   bits 0-8   neighbour POSITION, bit 9 OGS_SLOT_EDGE_DOWN (also for
   *              missing edges), bit 10 neighbour overloaded, bits 11-13
   *              rslot (reverse edge index in the neighbour's row),
   *   bits 16-31 metric.
   * Lets each lane load its edges coalesced straight into registers.
   * slot_degree is 4 or 8 (0 with slot_edges NULL). */
  const uint32_t* slot_edges;
  int32_t slot_degree;
  /* Optional [E_total] topology-local row (owner node) of every directed
   * edge: enables the edge-parallel multi-source path for topologies too
   * large for the wave kernel (all-sources batches, C3/C4/C5). */
  const uint32_t* edge_src;
  /* [E_total] exact reverse slot of every edge (the rslot field saturates at
   * 511). Required when any row has 512+ edges (max_degree >= 512): the KSP
   * path keys and link ids read it; optional (NULL) otherwise. */
  const uint32_t* rslot_ext;
} ogs_graph;

#define OGS_SLOT_EDGE_DOWN (1u << 9)
#define OGS_SLOT_EDGE_DST_OVERLOADED (1u << 10)
#define OGS_SLOT_EDGE_RSLOT_SHIFT 11

/* Prefix table: per topology a contiguous range of prefixes, each with a
 * contiguous segment of advertisements (one (node, area) entry each). */
typedef struct ogs_prefix_table {
  int32_t max_prefixes;       /* max prefixes of any topology (P stride) */
  int32_t max_advertisements; /* max advertisements of any topology      */
  const uint32_t* pfx_base;   /* [T+1] first global prefix of topology t */
  const uint32_t* adv_off;    /* [P_total+1] advertiser segment offsets  */
  const uint32_t* adv_node;   /* [A] local node id or OGS_NODE_NONE      */
  const int32_t* adv_metrics; /* [A*4] drain_metric, path_preference,
                                 source_preference, distance            */
  const int64_t* adv_min_nh;  /* [A] minNexthop, INT64_MIN when unset    */
  const uint8_t* pfx_flags;   /* [P_total] bit0: prefix is IPv4; bit1: an
                                 advertisement sets minNexthop           */
} ogs_prefix_table;

/* One work unit = (topology, source node). */
typedef struct ogs_unit {
  uint32_t topo;
  uint32_t src;
} ogs_unit;

/* Outputs (device). Any pointer may be NULL to skip that output. Layouts,
 * with U = unit index, S_n = graph.max_nodes, S_p = prefixes.max_prefixes,
 * W = nh_words:
 *   dist   [U*S_n + v]            uint32 (uint64 with OGS_F_WIDE_METRIC);
 *                                 all-ones = unreachable
 *   nh     [(U*W + w)*S_n + v]    link-slot bitset of node v
 *   meta   [U*S_p + p]            OGS_ROUTE_* flags | best << 8
 *   metric [U*S_p + p]            shortest metric (dist width)
 *   mask   [(U*W + w)*S_p + p]    next-hop link-slot bitset of the route
 *   sel    [U*S_p + p]            selected-advertiser bitset (segments of
 *                                 <= 32 entries; bestRoutesCache)
 *   reached [U*ceil(S_n/32) + v/32] bit v%32: node v settled. Written under
 *                                 OGS_F_EXACT_ORDER only, where a wrapped
 *                                 u64 distance of a reached node may be all
 *                                 ones (LinkState.cpp:77-78, 789); the other
 *                                 paths' distances never reach the sentinel */
typedef struct ogs_spf_out {
  void* dist;
  uint32_t* nh;
  uint32_t* meta;
  void* metric;
  uint32_t* mask;
  uint32_t* sel;
  uint32_t* reached;
} ogs_spf_out;

/* KSP2 unit: edge-disjoint paths src -> dest avoiding an optional
 * linksToIgnore mask. */
typedef struct ogs_path_unit {
  uint32_t topo;
  uint32_t src;
  uint32_t dest;
  uint32_t reserved;
} ogs_path_unit;

/* Paths (device). Per unit U: path_count[U] = number of paths (bit 31 set
 * if the output capacity was exceeded); path_len[U*max_paths + i] = links in
 * path i; path_edges[U*max_edges + ...] = the paths' topology-local directed
 * edge ids, concatenated, each path ordered source -> destination. */
typedef struct ogs_path_out {
  uint32_t* path_count;
  uint32_t* path_len;
  uint32_t* path_edges;
  uint32_t max_paths;
  uint32_t max_edges;
} ogs_path_out;

/* Multi-area routing domain (SpfSolver over several LinkStates, one per
 * area: SpfSolver.cpp:160-311). The areas are the
 * num_areas topologies of an ogs_graph batch; the domain has ONE prefix
 * table (ogs_prefix_table with num_topos = 1: pfx_base[0..1]) whose
 * advertisement segments list (node, area) entries in (node name, area
 * name) order, adv_node holding the node's id in ITS OWN area. Node names
 * are numbered across areas ("name ids") so the reference's by-name lookups
 * of selected advertisers in every area (SpfSolver.cpp:664-665) are one
 * table read. */
typedef struct ogs_area_table {
  int32_t num_areas;          /* A >= 1 (any number of areas)             */
  int32_t num_names;          /* G distinct node names of the domain      */
  const uint32_t* name_local; /* [G*A] id of name g in area a, or
                                 OGS_NODE_NONE if a has no such node     */
  const uint32_t* adv_area;   /* [A_total] area index of each entry       */
  const uint32_t* adv_name;   /* [A_total] name id of each entry's node   */
  /* Optional settled bitsets of the SPF rows ([row*ceil(S_n/32)], the
   * `reached` output of an OGS_F_EXACT_ORDER launch); NULL: all-ones
   * distance = unreachable. */
  const uint32_t* reached;
} ogs_area_table;

/* ---- runtime ------------------------------------------------------------ */
const char* ogs_version(void);
int ogs_abi_version(void); /* OGS_ABI_VERSION of the library */
const char* ogs_last_error(void); /* thread-local message of last failure */
int ogs_device_count(int* count);
int ogs_set_device(int device);
int ogs_malloc(void** dptr, size_t bytes);
int ogs_free(void* dptr);
int ogs_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int ogs_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int ogs_memset(void* dst, int value, size_t bytes, void* stream);
int ogs_stream_sync(void* stream);
/* Page-locked host memory (one DMA per transfer, no staging copy): the
 * adapter's per-call result blocks. */
int ogs_host_alloc(void** hptr, size_t bytes);
int ogs_host_free(void* hptr);

/* Tuning knobs of the DEFAULT context (the one the plain entry points use;
 * ogs_ctx_set_option sets a context's own copy; for A/B measurement):
 *   "unit_width": small-topology kernel choice: -1 automatic (default),
 *                 0 generic kernel only, 1 packed wave-per-unit kernel,
 *                 2 split-state kernel at its automatic unit width,
 *                 3 multi-source edge-parallel kernel (needs edge_src),
 *                 64 / 128 / 256 split-state kernel at that unit width.
 *   "wave_wg_lds": minimum LDS bytes per wave-kernel workgroup (occupancy
 *                 probe; 0 default). "wave_upb": units (wavefronts) per
 *                 wave-kernel workgroup, 4 (default), 8 or 16.
 *   "ms_group":   sources per workgroup of the multi-source kernel (0 auto,
 *                 1, 2, 4).
 *   "route_stream": RouteDb form for large shared topologies: 5 (default,
 *                 below; topologies whose LDS image does not fit take 2); 2
 *                 one launch per unit set, SPF then the unit's RouteDb write
 *                 stream from LDS; 1 an SPF launch then a route-stream launch
 *                 (dist/next-hop sets through HBM); 4 the SPF with the
 *                 topology staged in LDS, then the route stream over
 *                 "frontier_parts" workgroups per unit (A/B); 5 that SPF
 *                 and the stream in one persistent launch: "lds_grid"
 *                 workgroups (0 = one per CU) take SPF and stream items
 *                 ("lds_parts" prefix ranges per unit; 0, default: 2 when
 *                 every workgroup has 4+ units, else 4; "lds_tail" 1,
 *                 default: then the last grid's worth of units in 4) from a
 *                 device-wide counter, SPFs kept one grid ahead; route keys
 *                 packed into 16 bits on topologies of <= 16,384 nodes
 *                 ("lds_key16" 1, default; 0 u32 keys, A/B); on sharded
 *                 builds (fewer than 4 units per workgroup) the last grid's
 *                 worth of items in "lds_tail_parts" ranges per unit (0
 *                 auto: 2 x lds_parts) and "lds_lead" narrow units streamed
 *                 before the widest group (0, default: none; -1 a grid's
 *                 worth of items); unit-weight (BFS) SPFs stop once every
 *                 node is reached ("lds_bfs_exit" 1, default; 0 they run
 *                 the empty last layer, A/B) and pull a layer when 4 x the
 *                 unreached nodes' chunk records <= "lds_pull" x the
 *                 frontier's (6, default; 0 push only, A/B). Scratch
 *                 (prefix keys, dist/next-hop sets when out->dist / out->nh
 *                 are NULL) comes from a grow-only per-device workspace.
 *                 "route_store_nt", bits: 1 the RouteDb stream's 16-B stores
 *                 are non-temporal (else ordinary write-back stores), 2 the
 *                 wave kernel's output stores are; default 2 (A/B).
 *   "spf_packed_scan": 1 (default) chunk-scan frontier units with one-word
 *                 next-hop sets relax packed {dist, next hops} words in one
 *                 phase; 0 two phases (A/B). "spf_seed_row": 1 (default)
 *                 round 1 of the chunk scan relaxes the source's row
 *                 directly, 0 it scans every chunk record (A/B).
 *                 "spf_lane_walk": a round's active chunk records walked
 *                 per lane (1) or per batch slot (0); -1 (default) per lane
 *                 in workgroups of 512+ threads. "spf_preload": 1 (default)
 *                 the packed relax reads its 8 targets' distances before
 *                 any compare-and-swap, 0 not (A/B).
 *   "frontier_block": threads per workgroup of the all-sources RouteDb
 *                 launches (fused frontier SPF + route stream, meta / metric
 *                 / mask outputs): 256, 512 or 1024; 0 (default) by the
 *                 launch's streamed bytes per CU (256 for a whole-node
 *                 build, 512 for one rank's shard).
 *   "frontier_parts": workgroups per one-word unit of those launches, each
 *                 running the unit's SPF and streaming one prefix range
 *                 (1..16; 0 default: by bytes per CU). "frontier_parts_wide":
 *                 the same for units of wider next-hop sets.
 *   "wave_opt":   wave-kernel paths, bits: 1 register-resident SPF words
 *                 (ds_bpermute), 2 (default) identity-segment route path.
 *   "spf_frontier": 1 (default) large topologies (edge_src given) solve
 *                 SPF with the frontier kernel (one workgroup per unit,
 *                 only changed rows pushed); 0 the multi-source edge sweep.
 *   "spf_queue":  frontier kernel round schedule: -1 (default) LDS node
 *                 lists for sparse topologies (max degree <= 16; one phase
 *                 over packed {dist, next hops} words when the next-hop sets
 *                 fit one word), the chunk scan otherwise; 0 always the scan.
 *                 "spf_ninfo": 1 (default) the list forms keep row begin |
 *                 drained per node in LDS, 0 read them from the CSR, -1 the
 *                 CSR form whenever that raises the units per CU.
 *   "spf_global": 0 (default) units whose SPF state does not fit LDS
 *                 (tens of thousands of nodes) run the global-state path
 *                 (dist / next-hop sets / frontier lists in HBM, one 1024-
 *                 thread workgroup per unit, then one thread per route); 1
 *                 every ogs_spf_routes call takes that path (A/B, tests).
 *   "spf_global_sync": 1 (default) global-path rounds end with drained
 *                 stores + a barrier and state is read through L2-served
 *                 (sc1) loads; 0 agent-scope fences per round (A/B).
 *   "spf_global_lds": 1 (default) global-path distances and next-hop words
 *                 in LDS where both fit, else distances only; 2 distances
 *                 only; 0 all state in HBM (A/B).
 *   "ksp_hbm":    1 every KSP unit on the HBM-state path (A/B, tests); 0
 *                 (default) only units past LDS and OGS_F_EXACT_ORDER units.
 *                 "ksp_wave_trace": 1 (default) path traces of 32-bit
 *                 distance units run on a whole wavefront, 0 on one lane.
 *                 "ksp_prune": 1 (default) the KSP2 masked rerun skips and
 *                 does not queue nodes at or past the destination's current
 *                 distance (exact for metrics >= 1); 0 the full rerun (A/B).
 *   "c4_desc":    1 (default) the link-failure repair (OGS_F_INCREMENTAL)
 *                 seeds its affected set from precomputed descendant rows of
 *                 the base tight DAG (S_n <= 16384), 0 by growth rounds.
 *   "ksp_queue":  KSP2 batch SPF: 1 (default) LDS node lists, 0 the pull
 *                 fixpoint. "ksp_stage": -1 (default) auto, 0 CSR read
 *                 from HBM/L2, 1 row offsets in LDS, 2 rows + edges in LDS. */
int ogs_set_option(const char* name, int64_t value);

/* Smallest supported next-hop bitset width (words) for a source degree:
 * 1, 2, 4, 8 or 16 up to 512 links, ceil(degree / 32) past that (those
 * widths run the HBM-state kernels with a runtime word count). */
int ogs_nh_words_for_degree(int degree);

/* ---- compute ------------------------------------------------------------ *
 * Batched SPF (+ fused RouteDb when `prefixes` is non-NULL) for n_units
 * (topology, source) units, launched asynchronously on `stream` (a
 * hipStream_t; NULL = default stream). One wavefront per unit for small
 * topologies, one workgroup per unit for large ones (chosen internally).
 * 32-bit distances are exact only when max_metric * (max_nodes - 1) <
 * 2^31 - 1; the caller sets OGS_F_WIDE_METRIC otherwise (the adapter does).
 * Replaces: LinkState::runSpf/getSpfResult (LinkState.cpp:705-820) and the
 * per-prefix loop of SpfSolver::buildRouteDb (SpfSolver.cpp:335-340,
 * 160-311, 455-767), single area. */
int ogs_spf_routes(const ogs_graph* graph, const ogs_prefix_table* prefixes,
                   const ogs_unit* units /* device */, int32_t n_units,
                   uint32_t flags, int32_t nh_words, ogs_spf_out* out,
                   void* stream);

/* Several unit groups over ONE graph and prefix table, each with its own
 * next-hop width (nh_words) and outputs (out, by value, as ogs_spf_routes'
 * *out): the same results as one ogs_spf_routes call per group (a
 * BatchRunner's width groups, e.g. the C3 fabric's one- and three-word
 * sources), in as few launches as the engine can -- with "route_stream" 5
 * on a large shared topology one prep and ONE persistent launch for all
 * groups, so the widest group's SPFs and every group's route streams share
 * the CUs. groups: host array; groups with n_units == 0 are skipped. */
typedef struct ogs_route_group {
  const ogs_unit* units; /* device, n_units */
  int32_t n_units;
  int32_t nh_words;
  ogs_spf_out out;
} ogs_route_group;

int ogs_spf_routes_groups(const ogs_graph* graph, const ogs_prefix_table* prefixes,
                          const ogs_route_group* groups, int32_t n_groups, uint32_t flags,
                          void* stream);


/* RouteDb records of n_units units from SPF state a previous ogs_spf_routes
 * launch left in device memory (spf_dist [U*S_n] uint32, or uint64 with
 * OGS_F_WIDE_METRIC; spf_nh [(U*W + w)*S_n + v] link-slot sets; row u of the
 * state belongs to units[u]). One thread per (unit, prefix), route_one of
 * route_core.h. Replaces, for a prefix set whose SPF is already known, the
 * per-prefix createRouteForPrefix (SpfSolver.cpp:160-311) that
 * Decision::rebuildRoutes calls in its incremental branch (Decision.cpp:
 * 929-938): the SPF memo (LinkState::getSpfResult) reused, only the
 * changed prefixes routed. */
int ogs_routes_from_spf(const ogs_graph* graph, const ogs_prefix_table* prefixes,
                        const ogs_unit* units /* device */, int32_t n_units,
                        const void* spf_dist, const uint32_t* spf_nh,
                        const uint32_t* spf_reached /* optional, as out->reached */,
                        uint32_t flags, int32_t nh_words, ogs_spf_out* out,
                        void* stream);

/* Batched edge-disjoint path tracing (KSP2). For each unit: SPF from src
 * over the links not set in the unit's mask (`masks` + U*mask_words, bit l =
 * topology-local link id l = min of the link's two directed edge ids; NULL =
 * no mask), then the reference's greedy trace repeated until no path
 * remains. Replaces LinkState::getKthPaths / traceOnePath
 * (LinkState.cpp:226-247, 674-703): the k-th call is one launch whose masks
 * hold the links of the paths for 1..k-1. */
int ogs_ksp_paths(const ogs_graph* graph, const ogs_path_unit* units,
                  int32_t n_units, const uint32_t* masks, uint32_t mask_words,
                  uint32_t flags, ogs_path_out* out, void* stream);

/* Batched KSP2 (config C5): for each unit (topo, src, dest, reserved), the
 * paths of getKthPaths(src, dest, 1) into k1 and of getKthPaths(src, dest, 2)
 * into k2 (LinkState.cpp:674-703), in two launches on `stream`: one
 * unmasked SPF per entry of `sources` (device, n_sources (topo, src) pairs:
 * the memoised getSpfResult(src)), then per unit the k = 1 trace on that
 * SPF, a rerun with the k = 1 links ignored and the k = 2 trace. A unit's
 * `reserved` field is the index of its (topo, src) in `sources`; a unit
 * whose index is out of range or names another (topo, src) gets
 * path_count 0xC0000000 in both outputs. Distances of the sources live in
 * the per-device workspace. */
int ogs_ksp2_paths(const ogs_graph* graph, const ogs_unit* sources,
                   int32_t n_sources, const ogs_path_unit* units,
                   int32_t n_units, uint32_t flags, ogs_path_out* k1,
                   ogs_path_out* k2, void* stream);

/* Link-failure variants (config C4, the SURVEY §5 "link-flap variant"):
 * per unit, topology-local DIRECTED edge ids that are treated as removed --
 * the links an adjacency-database update deleted at both ends
 * (LinkState::updateAdjacencyDatabase, LinkState.cpp:491-634; list both
 * directions of each link). OGS_NODE_NONE pads a unit's list. Next-hop
 * link slots stay those of the unmodified CSR row, so a variant's records
 * compare slot for slot with the base's. */
typedef struct ogs_unit_mods {
  const uint32_t* dead_edges; /* [n_units * dead_per_unit]            */
  int32_t dead_per_unit;      /* 1..8                                  */
} ogs_unit_mods;

/* Route diff of every unit against ONE base unit's route records (same
 * topology, source and prefix table): DecisionRouteDb::calculateUpdate
 * (SpfSolver.cpp:21-56) with RibUnicastEntry::operator== (RibEntry.h:81-87):
 * a route is updated when it is new or its best entry (+ drain override),
 * local flag or next-hop set (metric and link mask) differ; igpCost and
 * bestArea are not compared. */
typedef struct ogs_route_diff {
  const uint32_t* base_meta;   /* [S_p]                                 */
  const uint32_t* base_metric; /* [S_p]                                 */
  const uint32_t* base_mask;   /* [W * S_p]                             */
  uint32_t* changed;           /* [n_units * ceil(S_p/32)] bit p set iff
                                  prefix p's route is added, updated or
                                  deleted (zeroed by the call)          */
  uint32_t* counts;            /* [n_units * 2] {routes to update,
                                  routes to delete}                     */
  const uint32_t* base_dist;   /* [S_n] base unit's distances and       */
  const uint32_t* base_nh;     /* [S_n] next-hop sets (ogs_spf_out of its
                                  ogs_spf_routes): OGS_F_INCREMENTAL    */
  /* [2 * A] optional: equality classes of the best entry a route would
   * carry -- adv_class[2a] for advertisement a as is, [2a + 1] with the
   * hard-drain override (drain_metric = 1); two routes' best entries are
   * equal (PrefixEntry ==, RibEntry.h:81-87) iff their classes are equal
   * (class = first position in the prefix's list [entries as is, entries
   * drained] holding an equal entry). NULL: compared by advertisement index
   * and DRAINED bit (a different but equal advertiser then counts as a
   * change). */
  const uint32_t* adv_class;
  /* Optional caller-held cache of the base unit's tight-DAG descendant rows
   * (OGS_F_INCREMENTAL repair; [S_n * ceil(S_n/32)] words, S_n <= 16384):
   * base_desc_valid == 0 -> the rows are computed into base_desc by this
   * call, 1 -> reused as they are. In / out: the call sets it to 1 when it
   * wrote the rows into base_desc and leaves it as it was otherwise (the
   * repair did not apply, or "c4_desc" is 0), so the caller keeps the
   * flag across calls. The rows depend only on the topology, the source
   * and the base SPF: the caller clears the flag when any of them changes
   * (the memo rule of LinkState.cpp:635-638). NULL: rebuilt in the
   * workspace on every call. */
  uint32_t* base_desc;
  int32_t base_desc_valid;
} ogs_route_diff;

/* Batched SPF + RouteDb of link-failure variants with an optional route
 * diff (mods / diff may be NULL). Large-topology path only (graph->edge_src
 * required, nh_words 1, 2 or 4, 32-bit distances); OGS_E_UNSUPPORTED
 * otherwise. Replaces, per variant, the reference's adjacency-DB update +
 * buildRouteDb + calculateUpdate. */
int ogs_spf_routes_variants(const ogs_graph* graph,
                            const ogs_prefix_table* prefixes,
                            const ogs_unit* units /* device */, int32_t n_units,
                            const ogs_unit_mods* mods,
                            ogs_route_diff* diff, uint32_t flags,
                            int32_t nh_words, ogs_spf_out* out, void* stream);

/* Compact list of the changed routes of n_units variants (SURVEY.md §8(f)
 * f1): what DecisionRouteDb::calculateUpdate (SpfSolver.cpp:21-56) hands
 * Fib through Decision::rebuildRoutes (Decision.cpp:929-951), gathered from
 * ogs_spf_routes_variants' records and changed bitmap. Unit-major, prefix
 * index ascending within a unit. A record whose meta lacks OGS_ROUTE_VALID
 * is a deletion (unicastRoutesToDelete), any other an update. */
typedef struct ogs_route_changes {
  const uint32_t* offsets; /* [n_units + 1] exclusive scan of each unit's
                              changed count (counts[2u] + counts[2u+1]);
                              offsets[n_units] == total                 */
  size_t total;            /* number of records (mask stride)           */
  uint32_t* prefix;        /* [total] prefix index in the unit's table  */
  uint32_t* meta;          /* [total] record meta (OGS_ROUTE_*)         */
  uint32_t* metric;        /* [total] route metric                      */
  uint32_t* mask;          /* [nh_words * total] link-slot mask, word w
                              of record i at mask[w * total + i]        */
} ogs_route_changes;

/* Gathers the changed records (diff->changed bitmap of the same call's
 * units, out->meta/metric/mask records of ogs_spf_routes_variants) into
 * `changes`. nh_words 1, 2 or 4 as for the variants call. */
int ogs_route_changes_gather(const uint32_t* changed, int32_t n_units,
                             int32_t max_prefixes, const ogs_spf_out* records,
                             int32_t nh_words, const ogs_route_changes* changes,
                             void* stream);

/* Incremental CSR update: edges[idx[i]] = val[i] for
 * i < n, idx / val device arrays (encoded as ogs_graph.edges). Replaces the
 * re-flatten + full re-upload after LinkState::updateAdjacencyDatabase
 * (LinkState.cpp:440-640) changed only link / node attributes (metric,
 * overload, usability): the CSR structure is unchanged. Indices must be
 * < the edge array's length (not checked on the device). */
int ogs_csr_patch(uint64_t* edges, const uint32_t* idx, const uint64_t* val,
                  int32_t n, void* stream);

/* RibPolicy compiled against one prefix table (SURVEY.md §8(a) a16;
 * RibPolicy.cpp:74-249): statements 0..K-1 in policy order. A policy of
 * more than 32 statements is applied as consecutive calls over chunks of
 * <= 32 (statement_base = 0, 32, 64, ...): a call with statement_base > 0
 * leaves the routes an earlier chunk transformed (applied !=
 * OGS_POLICY_NONE) as they are and continues the others' counter. Statement
 * indexes are u16 (OGS_POLICY_NONE = none): statement_base + K <= 65,535. */
#define OGS_POLICY_NONE 0xFFFFu /* applied / counter: no statement */

typedef struct ogs_rib_policy {
  int32_t num_statements;        /* K <= 32 (this chunk)                     */
  uint32_t active;               /* bit k: statement k has a prefix or tag
                                    matcher (no matcher never matches,
                                    RibPolicy.cpp:76-78)                    */
  const uint32_t* pfx_match;     /* [P_total] bit k: the prefix is in k's
                                    prefix set, or k has none                */
  const uint32_t* adv_tag_match; /* [A_total] bit k: the entry's tags meet
                                    k's tags, or k has none                 */
  const uint32_t* slot_nonzero;  /* [n_units][K][num_areas][W] link slots
                                    of the unit's source whose weight under
                                    statement k (neighbor > area > default,
                                    RibPolicy.cpp:122-137) is > 0           */
  int32_t statement_base;        /* policy index of this chunk's statement 0 */
} ogs_rib_policy;

/* Applies the policy to n_units RouteDbs in place (meta[U*S_p + p] read,
 * mask[((U*A + a)*W + w)*S_p + p] rewritten: next hops of weight 0 dropped
 * unless that drops all of them, RibPolicy.cpp:138-158). applied[U*S_p+p] =
 * statement whose weights the route took, counter[...] = statement whose
 * counterID the route carries (the last matching one tried), OGS_POLICY_NONE
 * = none. Statement ids are u16: a policy of up to 65,535 statements runs in
 * chunks of 32 (statement_base).
 * The prefix table is one topology's (pfx_base[0..1]); single-area callers
 * pass num_areas = 1. */
int ogs_rib_policy_apply(const ogs_prefix_table* prefixes,
                         const ogs_rib_policy* policy, int32_t num_areas,
                         int32_t n_units, int32_t nh_words,
                         const uint32_t* meta, uint32_t* mask,
                         uint16_t* applied, uint16_t* counter, void* stream);

/* Multi-area RouteDb for n_units sources from their per-area SPF results
 * (a prior ogs_spf_routes launch over the area batch without a prefix
 * table): units[u] = the source's name id; spf_row[u*A + a] = the row of
 * (source, area a) in spf_dist / spf_nh (layouts of ogs_spf_out with
 * S_n = graph->max_nodes and the same nh_words), OGS_NODE_NONE when the
 * source has no adjacency database in area a (its SPF there is the source
 * alone, LinkState.cpp:730-734). Outputs per unit as ogs_spf_out (meta,
 * metric, sel over S_p = prefixes->max_prefixes) with one next-hop mask per
 * area: mask[((U*A + a)*W + w)*S_p + p] over the source's links in area a.
 * spf_dist / out->metric are uint32, or uint64 with OGS_F_WIDE_METRIC (the
 * SPF launch's width, e.g. after OGS_F_EXACT_ORDER). Replaces createRouteForPrefix across areas
 * (SpfSolver.cpp:160-311: per-area reachability, selectBestRoutes 455-486,
 * areas with best routes, getNextHopsWithMetric per area 648-688, minimum
 * metric union over areas, addBestPaths 595-639). */
int ogs_routes_multiarea(const ogs_graph* graph,
                         const ogs_prefix_table* prefixes,
                         const ogs_area_table* areas,
                         const uint32_t* units /* device, [n_units] */,
                         int32_t n_units, const uint32_t* spf_row /* device */,
                         const void* spf_dist, const uint32_t* spf_nh,
                         uint32_t flags, int32_t nh_words, ogs_spf_out* out,
                         void* stream);

/* ---- execution contexts (ABI 6) ----------------------------------------- *
 * A context holds a device, its own copy of the tuning knobs (initialised
 * from the default context's at creation) and its own launch scratch (the
 * grow-only device workspace of the large-topology paths). The ogs_ctx_*
 * calls below take the same arguments as the plain entry points and run
 * them on the context's device with its knobs and scratch, so host threads
 * that each use their own context (and their own streams) never share
 * scratch or settings. A context is thread-compatible, not thread-safe: one
 * host thread at a time ("explicit stream/device handle;
 * thread-compatible, one context per host thread"). The plain entry points
 * keep using the process default context (scratch per (device, stream);
 * concurrent calls on ONE stream from several threads share it, so give
 * each thread its own context). Reference call sites: Decision's one
 * SpfSolver per Decision thread (Decision.cpp:912-913). */
typedef struct ogs_ctx ogs_ctx;
int ogs_ctx_create(int32_t device, ogs_ctx** out);
int ogs_ctx_destroy(ogs_ctx* ctx); /* waits for the device, frees the scratch */
int ogs_ctx_set_option(ogs_ctx* ctx, const char* name, int64_t value);
int ogs_ctx_spf_routes(ogs_ctx* ctx, const ogs_graph* graph, const ogs_prefix_table* prefixes,
                       const ogs_unit* units, int32_t n_units, uint32_t flags,
                       int32_t nh_words, ogs_spf_out* out, void* stream);
int ogs_ctx_spf_routes_groups(ogs_ctx* ctx, const ogs_graph* graph,
                              const ogs_prefix_table* prefixes, const ogs_route_group* groups,
                              int32_t n_groups, uint32_t flags, void* stream);
int ogs_ctx_routes_from_spf(ogs_ctx* ctx, const ogs_graph* graph,
                            const ogs_prefix_table* prefixes, const ogs_unit* units,
                            int32_t n_units, const void* spf_dist, const uint32_t* spf_nh,
                            const uint32_t* spf_reached, uint32_t flags, int32_t nh_words,
                            ogs_spf_out* out, void* stream);
int ogs_ctx_spf_routes_variants(ogs_ctx* ctx, const ogs_graph* graph,
                                const ogs_prefix_table* prefixes, const ogs_unit* units,
                                int32_t n_units, const ogs_unit_mods* mods,
                                ogs_route_diff* diff, uint32_t flags, int32_t nh_words,
                                ogs_spf_out* out, void* stream);
int ogs_ctx_ksp_paths(ogs_ctx* ctx, const ogs_graph* graph, const ogs_path_unit* units,
                      int32_t n_units, const uint32_t* masks, uint32_t mask_words,
                      uint32_t flags, ogs_path_out* out, void* stream);
int ogs_ctx_ksp2_paths(ogs_ctx* ctx, const ogs_graph* graph, const ogs_unit* sources,
                       int32_t n_sources, const ogs_path_unit* units, int32_t n_units,
                       uint32_t flags, ogs_path_out* k1, ogs_path_out* k2, void* stream);
int ogs_ctx_routes_multiarea(ogs_ctx* ctx, const ogs_graph* graph,
                             const ogs_prefix_table* prefixes, const ogs_area_table* areas,
                             const uint32_t* units, int32_t n_units, const uint32_t* spf_row,
                             const void* spf_dist, const uint32_t* spf_nh, uint32_t flags,
                             int32_t nh_words, ogs_spf_out* out, void* stream);
int ogs_ctx_rib_policy_apply(ogs_ctx* ctx, const ogs_prefix_table* prefixes,
                             const ogs_rib_policy* policy, int32_t num_areas, int32_t n_units,
                             int32_t nh_words, const uint32_t* meta, uint32_t* mask,
                             uint16_t* applied, uint16_t* counter, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OPENR_GPU_H_ */
