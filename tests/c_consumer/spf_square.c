/* A plain-C consumer of the drop-in boundary (include/openr_gpu.h): what a
 * cgo / JNI / ctypes binding does underneath. Builds a 4-node topology in the
 * C-ABI's CSR encoding, runs ogs_spf_routes from node 0 with no prefix table
 * and checks distances and ECMP next-hop link slots.
 *   0 --1-- 1 --1-- 2 --1-- 3,   0 --2-- 2,   0 --5-- 3
 * From 0: dist {0, 1, 2, 3}; 2 is reached through 1 and directly (ECMP: link
 * slots 0 and 1 of node 0), 3 through 2 (same set).
 * Exit status: 0 ok, 77 no HIP device (skip), 1 mismatch, 2 C-ABI error. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "openr_gpu.h"

static uint64_t edge(uint32_t dst, uint32_t rslot, uint32_t w) {
  return (uint64_t)(dst | (rslot << OGS_EDGE_RSLOT_SHIFT)) | ((uint64_t)w << 32);
}

#define CHECK(x)                                                   \
  do {                                                             \
    int rc_ = (x);                                                 \
    if (rc_ != OGS_OK) {                                           \
      fprintf(stderr, "%s -> %d: %s\n", #x, rc_, ogs_last_error()); \
      return 2;                                                    \
    }                                                              \
  } while (0)

int main(void) {
  int devices = 0;
  if (ogs_device_count(&devices) != OGS_OK || devices <= 0) {
    printf("no HIP device\n");
    return 77;
  }
  /* rows: 0 -> {1, 2, 3}, 1 -> {0, 2}, 2 -> {0, 1, 3}, 3 -> {0, 2} */
  const uint32_t node_base[2] = {0, 4};
  const uint32_t row_ptr[5] = {0, 3, 5, 8, 10};
  const uint64_t edges[10] = {
      edge(1, 0, 1), edge(2, 0, 2), edge(3, 0, 5),  /* node 0 */
      edge(0, 0, 1), edge(2, 1, 1),                 /* node 1 */
      edge(0, 1, 2), edge(1, 1, 1), edge(3, 1, 1),  /* node 2 */
      edge(0, 2, 5), edge(2, 2, 1)};                /* node 3 */
  const uint8_t flags[4] = {0, 0, 0, 0};
  const ogs_unit unit = {0, 0};
  void *d_nb, *d_row, *d_edges, *d_flags, *d_unit, *d_dist, *d_nh;
  CHECK(ogs_malloc(&d_nb, sizeof node_base));
  CHECK(ogs_malloc(&d_row, sizeof row_ptr));
  CHECK(ogs_malloc(&d_edges, sizeof edges));
  CHECK(ogs_malloc(&d_flags, sizeof flags));
  CHECK(ogs_malloc(&d_unit, sizeof unit));
  CHECK(ogs_malloc(&d_dist, 4 * sizeof(uint32_t)));
  CHECK(ogs_malloc(&d_nh, 4 * sizeof(uint32_t)));
  CHECK(ogs_memcpy_h2d(d_nb, node_base, sizeof node_base, NULL));
  CHECK(ogs_memcpy_h2d(d_row, row_ptr, sizeof row_ptr, NULL));
  CHECK(ogs_memcpy_h2d(d_edges, edges, sizeof edges, NULL));
  CHECK(ogs_memcpy_h2d(d_flags, flags, sizeof flags, NULL));
  CHECK(ogs_memcpy_h2d(d_unit, &unit, sizeof unit, NULL));

  if (ogs_abi_version() != OGS_ABI_VERSION) {  /* header and library agree */
    fprintf(stderr, "ABI %d, header %d\n", ogs_abi_version(), OGS_ABI_VERSION);
    return 2;
  }
  ogs_graph g;
  memset(&g, 0, sizeof g);
  g.num_topos = 1;
  g.max_nodes = 4;
  g.max_edges = 10;
  g.max_degree = 3;
  g.node_base = (const uint32_t*)d_nb;
  g.row_ptr = (const uint32_t*)d_row;
  g.edges = (const uint64_t*)d_edges;
  g.node_flags = (const uint8_t*)d_flags;
  ogs_spf_out out;
  memset(&out, 0, sizeof out);
  out.dist = d_dist;
  out.nh = (uint32_t*)d_nh;
  CHECK(ogs_spf_routes(&g, NULL, (const ogs_unit*)d_unit, 1, 0, 1, &out, NULL));
  uint32_t dist[4], nh[4];
  CHECK(ogs_memcpy_d2h(dist, d_dist, sizeof dist, NULL));
  CHECK(ogs_memcpy_d2h(nh, d_nh, sizeof nh, NULL));
  CHECK(ogs_stream_sync(NULL));
  const uint32_t want_dist[4] = {0, 1, 2, 3};
  const uint32_t want_nh[4] = {0, 0x1, 0x3, 0x3};
  int bad = 0;
  for (int v = 0; v < 4; ++v) {
    printf("node %d: dist %u nh 0x%x\n", v, dist[v], nh[v]);
    bad |= dist[v] != want_dist[v] || nh[v] != want_nh[v];
  }
  /* the same SPF through an execution context (ABI 6) with its own knobs */
  ogs_ctx* ctx = NULL;
  CHECK(ogs_ctx_create(0, &ctx));
  CHECK(ogs_ctx_set_option(ctx, "unit_width", 0)); /* the generic kernel, this context only */
  CHECK(ogs_memset(d_dist, 0xFF, sizeof dist, NULL));
  CHECK(ogs_ctx_spf_routes(ctx, &g, NULL, (const ogs_unit*)d_unit, 1, 0, 1, &out, NULL));
  CHECK(ogs_memcpy_d2h(dist, d_dist, sizeof dist, NULL));
  CHECK(ogs_memcpy_d2h(nh, d_nh, sizeof nh, NULL));
  CHECK(ogs_stream_sync(NULL));
  CHECK(ogs_ctx_destroy(ctx));
  for (int v = 0; v < 4; ++v) bad |= dist[v] != want_dist[v] || nh[v] != want_nh[v];
  printf("context: %s\n", bad ? "MISMATCH" : "ok");
  ogs_free(d_nb);
  ogs_free(d_row);
  ogs_free(d_edges);
  ogs_free(d_flags);
  ogs_free(d_unit);
  ogs_free(d_dist);
  ogs_free(d_nh);
  return bad ? 1 : 0;
}
