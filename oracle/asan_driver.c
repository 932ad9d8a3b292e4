/* asan_driver.c — runs every entry point of the C oracle on small inputs so
 * that a build with -fsanitize=address,undefined (tests/test_oracle_asan.py
 * compiles it with hz_oracle.c) reports any out-of-bounds access, leak,
 * undefined shift or signed overflow in the restatement (the C
 * restatement under ASan/UBSan).  TEST INFRASTRUCTURE ONLY: built and run
 * by tests/test_oracle_asan.py on the CPU; prints "asan driver ok" and a
 * checksum of what it computed. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hz_oracle.h"

static uint64_t mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  return h;
}

int main(void) {
  uint64_t h = 0;
  enum { N = 48 };
  int16_t finals[N * OR_REFSTATE];
  int32_t plies[N], games[N], ep[N], rejected[N];
  uint32_t nxt[N];

  /* whole rule games, two episodes, and the auto-reset restatement */
  h = mix(h, (uint64_t)or_play_rule_games(N, 11, finals, plies, nxt, 1));
  for (int i = 0; i < N; i++) h = mix(h, (uint64_t)(plies[i] * 131 + finals[i * OR_REFSTATE + 76]) ^ nxt[i]);
  h = mix(h, (uint64_t)or_play_rule_games_ep(N, 11, 3, finals, plies, nxt, 1));
  h = mix(h, (uint64_t)or_play_rule_auto(N, 5, 0, 250, finals, games, ep, 1));
  for (int i = 0; i < N; i++) h = mix(h, (uint64_t)(games[i] * 7 + ep[i]));

  /* a caller's own moves, legal and not (rejected moves leave the board) */
  enum { P = 90 };
  uint64_t seeds[N];
  int16_t *acts = (int16_t *)malloc(sizeof(int16_t) * P * N);
  for (int b = 0; b < N; b++) seeds[b] = 1000 + (uint64_t)b;
  uint64_t r = 12345;
  for (int k = 0; k < P * N; k++) {
    r = r * 6364136223846793005ull + 1442695040888963407ull;
    acts[k] = (int16_t)((int)(r >> 33) % 150) - 3;  /* -3 .. 146: no-ops, legal, illegal, out of range */
  }
  h = mix(h, (uint64_t)or_replay_actions(N, seeds, P, acts, finals, rejected, 1));
  for (int i = 0; i < N; i++) h = mix(h, (uint64_t)rejected[i]);
  free(acts);

  /* one game by hand: legal masks, every encoder, canonical keys, scoring,
   * greedy moves and searches along it */
  or_mt m, g;
  int16_t st[OR_REFSTATE];
  uint8_t mask[143], key[128], cells[23];
  float board[1330], glob[42], pol[143];
  double v, noise[143];
  int32_t visits[143], nn, ne, parts[5];
  for (int i = 0; i < 143; i++) noise[i] = 1.0 / 143;
  or_mt_seed(&m, 777);
  or_reset(&m, st);
  for (int ply = 0; ply < 200 && !or_is_game_over(st); ply++) {
    const int L = or_legal(st, mask);
    or_encode(st, board, glob);
    or_canonical(st, key, ply & 1);
    or_stub_eval(st, pol, &v);
    for (int p = 0; p < 2; p++) {
      for (int c = 0; c < 23; c++) cells[c] = (uint8_t)st[23 * p + c];
      or_score_board(cells, parts);
      for (int k = 0; k < 5; k++) h = mix(h, (uint64_t)parts[k]);
    }
    for (int i = 0; i < 128; i++) h = mix(h, key[i]);
    h = mix(h, (uint64_t)(int64_t)(board[ply % 1330] * 64) ^ (uint64_t)(int64_t)(glob[ply % 42] * 64));
    if (ply % 9 == 0) {
      memcpy(&g, &m, sizeof g);
      h = mix(h, (uint64_t)or_greedy_move(st, &g));
      or_mcts_cfg cfg = {16, 1.0f, 0.25, ply & 1, 10, ply, 0.5, ply % 2, ply % 3 == 0};
      memcpy(&g, &m, sizeof g);
      const int a = or_mcts_search(st, &g, &cfg, noise, visits, &nn, &ne);
      h = mix(h, (uint64_t)(a + 7 * nn + 11 * ne));
      for (int i = 0; i < 143; i++) h = mix(h, (uint64_t)visits[i]);
    }
    int a = -1, k = (int)(or_rule(777, (uint64_t)ply) >> 32) % (L > 0 ? L : 1);
    for (int i = 0; i < 143 && a < 0; i++)
      if (mask[i] && k-- == 0) a = i;
    if (a < 0) break;
    h = mix(h, (uint64_t)or_step(st, a, &m));
    h = mix(h, (uint64_t)or_step(st, 142, &m) + 1);  /* usually illegal: a status, the board unchanged */
  }
  for (int i = 0; i < 4; i++) h = mix(h, or_randbelow(&m, 1 + 37u * (uint32_t)i));
  int32_t smp[8];
  or_sample(&m, 40, 8, smp);
  for (int i = 0; i < 8; i++) h = mix(h, (uint64_t)smp[i]);
  printf("asan driver ok %016llx\n", (unsigned long long)h);
  return 0;
}
