/* Host-code sanitizer driver (CPU test, tests/test_host.py::test_host_code_under_asan).
 *
 * Linked against libmev_asan.so (`make asan`: the host side compiled with
 * -Xarch_host -fsanitize=address,undefined, the gfx950 device code built as usual and never
 * launched here -- there is no GPU in the container), it calls every C-ABI entry point that does host
 * work without a GPU -- argument checks, numpy-compatible seeding, the libm channel table,
 * mev_create's validation and its failure path -- with buffers sized exactly, so an
 * out-of-bounds write or undefined behaviour in the host code aborts the run. Prints the seed
 * rows and the table's first entries for the Python side to compare with numpy / the oracle. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mev.h"

#define CHECK(cond)                                                  \
  do {                                                               \
    if (!(cond)) {                                                   \
      fprintf(stderr, "check failed: %s (line %d)\n", #cond, __LINE__); \
      return 1;                                                      \
    }                                                                \
  } while (0)

static void defaults(mev_params* p) {
  memset(p, 0, sizeof(*p));
  p->num_envs = 4;
  p->num_ues = 30;
  p->num_bs = 13;
  p->width = 200;
  p->height = 200;
  p->ep_max_time = 20;
  p->arrival_exit = 20;
  p->first_step_active = 1;
  p->movement_reseed = 1;
  p->draw_table = -1;
  p->velocity = 1.5;
  p->bs_bw = 9e6;
  p->bs_freq = 2500;
  p->bs_tx = 40;
  p->bs_height = 50;
  p->ue_snr_tr = 2e-8;
  p->ue_noise = 1e-9;
  p->ue_height = 1.6;
  p->util_lower = -20;
  p->util_upper = 20;
  p->util_w1 = 10;
  p->util_w2 = 0;
  p->util_w3 = 10;
}

int main(void) {
  CHECK(mev_abi_version() == MEV_ABI_VERSION);
  const int codes[] = {MEV_OK, MEV_EINVAL, MEV_ENOMEM, MEV_EHIP, MEV_ECHANNEL, 12345, -7};
  for (size_t i = 0; i < sizeof(codes) / sizeof(codes[0]); ++i) CHECK(mev_strerror(codes[i]) != NULL);
  CHECK(mev_last_hip_error() != NULL);

  /* seeding: empty, invalid, three seeds into an exactly sized heap buffer */
  CHECK(mev_seed_pcg64(NULL, 0, NULL) == MEV_OK);
  CHECK(mev_seed_pcg64(NULL, 2, NULL) == MEV_EINVAL);
  const uint64_t bad[1] = {1ull << 63};
  uint64_t* one = (uint64_t*)malloc(6 * sizeof(uint64_t));
  CHECK(mev_seed_pcg64(bad, 1, one) == MEV_EINVAL);
  free(one);
  const uint64_t seeds[3] = {0, 1004, (1ull << 63) - 1};
  uint64_t* rows = (uint64_t*)malloc(3 * 6 * sizeof(uint64_t));
  CHECK(mev_seed_pcg64(seeds, 3, rows) == MEV_OK);
  for (int i = 0; i < 3; ++i)
    printf("seed %llu %llu %llu %llu %llu\n", (unsigned long long)seeds[i],
           (unsigned long long)rows[6 * i], (unsigned long long)rows[6 * i + 1],
           (unsigned long long)rows[6 * i + 2], (unsigned long long)rows[6 * i + 3]);
  free(rows);

  /* channel table: argument checks, query, a short prefix, the whole table */
  mev_params p;
  defaults(&p);
  CHECK(mev_build_rate_table(NULL, NULL, 0) == MEV_EINVAL);
  CHECK(mev_build_rate_table(&p, NULL, 5) == MEV_EINVAL);
  CHECK(mev_build_rate_table(&p, NULL, -1) == MEV_EINVAL);
  const int64_t n = mev_build_rate_table(&p, NULL, 0);
  CHECK(n > 1000);
  double* head = (double*)malloc(7 * sizeof(double));
  CHECK(mev_build_rate_table(&p, head, 7) == n);
  double* tab = (double*)malloc((size_t)n * sizeof(double));
  CHECK(mev_build_rate_table(&p, tab, n) == n);
  CHECK(memcmp(head, tab, 7 * sizeof(double)) == 0);
  printf("table %lld %.17g %.17g %.17g\n", (long long)n, tab[1], tab[n / 2], tab[n - 1]);
  free(head);
  free(tab);
  mev_params q = p;
  q.width = 0;
  CHECK(mev_build_rate_table(&q, NULL, 0) == MEV_EINVAL);
  q = p;
  q.width = 1024;
  q.height = 1024;
  CHECK(mev_build_rate_table(&q, NULL, 0) == n);  /* reach ends inside the map either way */

  /* mev_create: validation, then (no device code / no GPU here) a failure that must release
   * the partly built context */
  mev_ctx* ctx = (mev_ctx*)0x1;
  CHECK(mev_create(&p, NULL) == MEV_EINVAL);
  q = p;
  q.num_ues = 0;
  CHECK(mev_create(&q, &ctx) == MEV_EINVAL && ctx == NULL);
  q = p;
  q.num_bs = 100000;
  CHECK(mev_create(&q, &ctx) == MEV_EINVAL && ctx == NULL);
  const int rc = mev_create(&p, &ctx);
  if (rc == MEV_OK) mev_destroy(ctx);
  else CHECK(ctx == NULL);
  printf("create %d\n", rc);
  mev_destroy(NULL);
  printf("ok\n");
  return 0;
}
