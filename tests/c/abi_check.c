/* C99 consumer of include/wats_hip.h: the boundary is plain C (no torch or
 * C++ types).  Built and run by tests/test_host.py without a GPU: only the
 * calls that validate their arguments before any device work are made. */
#include <stdio.h>
#include <string.h>

#include "wats_hip.h"

int main(void) {
  wg_laplacian_t L = NULL;
  int rc;
  if (wg_abi_version() != WG_ABI_VERSION) {
    fprintf(stderr, "abi version %d != %d\n", wg_abi_version(), WG_ABI_VERSION);
    return 1;
  }
  rc = wg_laplacian_create(-1, 0, 0, NULL, NULL, NULL, NULL, WG_FLAG_NONE, NULL, &L);
  if (rc != WG_ERR_INVALID || L != NULL || strstr(wg_last_error(), "bad shape") == NULL) {
    fprintf(stderr, "create: rc=%d msg=%s\n", rc, wg_last_error());
    return 2;
  }
  rc = wg_wavelet_features(NULL, NULL, 1, 3, 0.8, NULL, NULL, NULL);
  if (rc != WG_ERR_INVALID) return 3;
  rc = wg_dist_create(NULL, NULL, 0, 1, NULL, NULL, NULL, NULL);
  if (rc != WG_ERR_INVALID) return 4;
  printf("ok %s\n", wg_last_error());
  return 0;
}
