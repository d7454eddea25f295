/* A minimal stand-in for an MPI library (MPICH ABI: integer handles) used by
 * tests/test_network.py to drive src/network/mpi_transport.cpp without an MPI installation.
 * Ranks are separate processes: FAKE_MPI_RANK / FAKE_MPI_SIZE give the rank and world size,
 * FAKE_MPI_DIR a directory shared by all of them.  A message is a file written under a
 * temporary name and renamed into place (m_<src>_<dst>_<seq>); the receiver polls for it,
 * reads and deletes it.  Sends therefore never block, so Sendrecv and Allgatherv cannot
 * deadlock.  Only the calls the transport makes are implemented.
 *
 *   gcc -shared -fPIC -O1 -o libfakempi.so fake_mpi.c
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#define MAX_RANKS 64

static int g_init = 0, g_fin = 0, g_rank = -1, g_size = 0;
static const char* g_dir = NULL;
static unsigned long g_send_seq[MAX_RANKS], g_recv_seq[MAX_RANKS];

static void setup(void) {
  if (g_rank >= 0) return;
  const char* r = getenv("FAKE_MPI_RANK");
  const char* s = getenv("FAKE_MPI_SIZE");
  g_dir = getenv("FAKE_MPI_DIR");
  g_rank = r ? atoi(r) : 0;
  g_size = s ? atoi(s) : 1;
  if (!g_dir) g_dir = "/tmp";
}

static int put(int dst, const void* buf, int len) {
  char tmp[512], fin[512];
  const unsigned long seq = g_send_seq[dst]++;
  snprintf(tmp, sizeof tmp, "%s/t_%d_%d_%lu", g_dir, g_rank, dst, seq);
  snprintf(fin, sizeof fin, "%s/m_%d_%d_%lu", g_dir, g_rank, dst, seq);
  FILE* f = fopen(tmp, "wb");
  if (!f) return 1;
  if (len > 0 && fwrite(buf, 1, (size_t)len, f) != (size_t)len) {
    fclose(f);
    return 2;
  }
  fclose(f);
  return rename(tmp, fin) == 0 ? 0 : 3;
}

static int get(int src, void* buf, int len) {
  char fin[512];
  const unsigned long seq = g_recv_seq[src]++;
  snprintf(fin, sizeof fin, "%s/m_%d_%d_%lu", g_dir, src, g_rank, seq);
  struct stat st;
  const time_t t0 = time(NULL);
  while (stat(fin, &st) != 0) {
    if (time(NULL) - t0 > 60) return 4; /* the peer never sent: an error, not a hang */
    usleep(200);
  }
  if (st.st_size != len) return 5;
  FILE* f = fopen(fin, "rb");
  if (!f) return 6;
  if (len > 0 && fread(buf, 1, (size_t)len, f) != (size_t)len) {
    fclose(f);
    return 7;
  }
  fclose(f);
  unlink(fin);
  return 0;
}

int MPI_Initialized(int* flag) {
  *flag = g_init;
  return 0;
}
int MPI_Finalized(int* flag) {
  *flag = g_fin;
  return 0;
}
int MPI_Init_thread(int* argc, char*** argv, int required, int* provided) {
  (void)argc;
  (void)argv;
  setup();
  g_init = 1;
  *provided = required;
  return 0;
}
int MPI_Comm_size(int comm, int* size) {
  if (comm != 0x44000000) return 10;
  *size = g_size;
  return 0;
}
int MPI_Comm_rank(int comm, int* rank) {
  if (comm != 0x44000000) return 10;
  *rank = g_rank;
  return 0;
}
int MPI_Sendrecv(const void* sbuf, int scount, int stype, int dst, int stag, void* rbuf, int rcount, int rtype, int src,
                 int rtag, int comm, void* status) {
  (void)stag;
  (void)rtag;
  (void)status;
  if (stype != 0x4c00010d || rtype != 0x4c00010d || comm != 0x44000000) return 11;
  int rc = put(dst, sbuf, scount);
  return rc ? rc : get(src, rbuf, rcount);
}
int MPI_Allgatherv(const void* sbuf, int scount, int stype, void* rbuf, const int* rcounts, const int* displs, int rtype,
                   int comm) {
  if (stype != 0x4c00010d || rtype != 0x4c00010d || comm != 0x44000000) return 11;
  if (scount != rcounts[g_rank]) return 12;
  memcpy((char*)rbuf + displs[g_rank], sbuf, (size_t)scount);
  for (int r = 0; r < g_size; ++r) {
    if (r != g_rank && put(r, sbuf, scount)) return 13;
  }
  for (int r = 0; r < g_size; ++r) {
    if (r != g_rank) {
      int rc = get(r, (char*)rbuf + displs[r], rcounts[r]);
      if (rc) return rc;
    }
  }
  return 0;
}
int MPI_Barrier(int comm) {
  char z = 0;
  int counts[MAX_RANKS] = {0}, displs[MAX_RANKS] = {0};
  (void)z;
  return MPI_Allgatherv(&z, 0, 0x4c00010d, &z, counts, displs, 0x4c00010d, comm);
}
int MPI_Finalize(void) {
  g_fin = 1;
  FILE* f;
  char p[512];
  snprintf(p, sizeof p, "%s/finalized_%d", g_dir, g_rank);
  f = fopen(p, "w");
  if (f) fclose(f);
  return 0;
}
int MPI_Abort(int comm, int code) {
  (void)comm;
  _exit(code == 0 ? 1 : code & 0xff);
}
