/*
 * tests/golden/config1_runner.c -- TEST INFRASTRUCTURE ONLY (fixture generator helper).
 *
 * Runs an afl-gcc-instrumented target once per input and captures its RAW 8-bit hit counters,
 * the way the reference's AFL plugin sees them before finish_fuzz_round
 * (instrumentation/afl_instrumentation.c:153-180 enable -> setup_shm/memset, :231-274): a SysV
 * SHM map of MAP_SIZE bytes named by __AFL_SHM_ID (afl_progs/config.h:267), cleared before every
 * exec, the input on the target's stdin (the stdin driver, tests/smoke_test.sh:164).  There is
 * no fork server: the target's trampoline sees fd 199 closed and runs normally
 * (afl_progs/afl-as.h __afl_forkserver: "If this fails, assume ... the parent doesn't want to
 * use the fork server").  Outcome per exec: 0 = exit (FUZZ_NONE), 1 = timeout (FUZZ_HANG),
 * 2 = signal (FUZZ_CRASH).
 *
 * usage: config1_runner <target> <inputs.bin> <n> <len> <out_maps.bin> <out_outcomes.bin>
 *   inputs.bin: n inputs of len bytes each; out_maps.bin: n x 65536 bytes.
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ipc.h>
#include <sys/shm.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#define MAP_SIZE 65536

int main(int argc, char **argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s target inputs n len maps outcomes\n", argv[0]);
    return 2;
  }
  const char *target = argv[1];
  const long n = atol(argv[3]), len = atol(argv[4]);
  FILE *fi = fopen(argv[2], "rb"), *fm = fopen(argv[5], "wb"), *fo = fopen(argv[6], "wb");
  if (!fi || !fm || !fo) return 2;
  const int shm_id = shmget(IPC_PRIVATE, MAP_SIZE, IPC_CREAT | IPC_EXCL | 0600);
  if (shm_id < 0) return 3;
  unsigned char *map = shmat(shm_id, NULL, 0);
  if (map == (void *)-1) return 3;
  char id[32];
  snprintf(id, sizeof(id), "%d", shm_id);
  setenv("__AFL_SHM_ID", id, 1);
  unsigned char *in = malloc(len);
  int rc = 0;
  for (long j = 0; j < n && !rc; j++) {
    if (fread(in, 1, len, fi) != (size_t)len) { rc = 4; break; }
    memset(map, 0, MAP_SIZE);
    int p[2];
    if (pipe(p)) { rc = 5; break; }
    const pid_t pid = fork();
    if (pid == 0) {
      dup2(p[0], 0);
      close(p[0]);
      close(p[1]);
      const int dn = open("/dev/null", 1);
      if (dn >= 0) { dup2(dn, 1); dup2(dn, 2); }
      execl(target, target, (char *)NULL);
      _exit(127);
    }
    close(p[0]);
    if (write(p[1], in, len) != len) { /* target may exit early */ }
    close(p[1]);
    int status = 0;
    signed char oc = 0;
    for (int waited = 0;; waited++) {  /* 2 s timeout, polled every ms */
      const pid_t r = waitpid(pid, &status, WNOHANG);
      if (r == pid) break;
      if (waited >= 2000) {
        kill(pid, SIGKILL);
        waitpid(pid, &status, 0);
        oc = 1;
        break;
      }
      usleep(1000);
    }
    if (!oc && WIFSIGNALED(status)) oc = 2;
    if (!oc && WIFEXITED(status) && WEXITSTATUS(status) == 127) { rc = 6; break; }
    fwrite(map, 1, MAP_SIZE, fm);
    fwrite(&oc, 1, 1, fo);
  }
  shmdt(map);
  shmctl(shm_id, IPC_RMID, NULL);
  fclose(fi);
  fclose(fm);
  fclose(fo);
  return rc;
}
