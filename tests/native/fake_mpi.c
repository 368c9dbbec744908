/* Test double of an MPICH-ABI MPI (MPI_Comm = int, MPI_BYTE = 0x4c00010d) for the bridge's
 * ncclUniqueId bootstrap (csrc/bridge.hip share_unique_id): rank and size from
 * FAKE_MPI_RANK / FAKE_MPI_SIZE, MPI_Bcast from root 0 through a file in FAKE_MPI_DIR.
 * Every call is logged to FAKE_MPI_DIR/log.<rank> so the test can check the handle and
 * datatype the bridge passed.  Loaded RTLD_GLOBAL before the bridge library. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static void logf_(const char* what, long a, long b) {
  char p[512];
  snprintf(p, sizeof p, "%s/log.%s", getenv("FAKE_MPI_DIR"), getenv("FAKE_MPI_RANK"));
  FILE* f = fopen(p, "a");
  fprintf(f, "%s %ld %ld\n", what, a, b);
  fclose(f);
}

int MPI_Initialized(int* flag) { *flag = 1; return 0; }
int MPI_Comm_f2c(int h) { logf_("f2c", h, 0); return h; }
int MPI_Comm_rank(int c, int* r) { *r = atoi(getenv("FAKE_MPI_RANK")); logf_("rank", c, *r); return 0; }
int MPI_Comm_size(int c, int* s) { *s = atoi(getenv("FAKE_MPI_SIZE")); logf_("size", c, *s); return 0; }

int MPI_Bcast(void* buf, int n, int type, int root, int comm) {
  char p[512], tmp[520];
  snprintf(p, sizeof p, "%s/bcast.%d", getenv("FAKE_MPI_DIR"), comm);
  logf_("bcast", comm, (long)type * 1000 + n);
  if (type != 0x4c00010d || root != 0) return 1;
  if (atoi(getenv("FAKE_MPI_RANK")) == 0) {
    snprintf(tmp, sizeof tmp, "%s.tmp", p);
    FILE* f = fopen(tmp, "wb");
    fwrite(buf, 1, n, f);
    fclose(f);
    rename(tmp, p);
    return 0;
  }
  for (int t = 0; t < 3000; ++t) {
    FILE* f = fopen(p, "rb");
    if (f) {
      size_t got = fread(buf, 1, n, f);
      fclose(f);
      if ((int)got == n) return 0;
    }
    usleep(10000);
  }
  return 2;
}
