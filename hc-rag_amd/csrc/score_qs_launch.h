// score_qs_launch.h — host interface of the query-stationary score kernel (score_qs.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

struct QsArgs {
  const void* rows;          // corpus rows, storage dtype (f16 / bf16), [n + slack][ld]
  int ld;
  int64_t n_rows;
  const float* inv32;
  const uint32_t* mask;      // row bitmask or nullptr
  const void* qhat;          // unit queries, MFMA dtype, [nqb * 128 * nq_blocks][ld]
  int nqb, P, ntiles, tstride;
  uint64_t* buf;             // [nqb * P][QT][cap] candidate buffers
  uint32_t* tau_g;
  uint64_t* partials;        // [q][P x kp] append regions (final_list)
  int* pcnt;                 // [q] append counters
  int kp;
  int cap;                   // qs_cap(kp)
  bool unit;                 // raw dot products as coarse scores (L2-normalised corpus)
  int nq_blocks;             // 16-query blocks per wave: 1 (256-row tiles) or 2 (128-row tiles)
  int hs = 2;                // 32-deep k-steps per ring stage (2; 4 for the 256-query form at
                             // KS = 12)
  float* umax = nullptr;     // QW: the MAXONLY sampling pre-pass into umax[unit][nqb * 256]
                             // (ntiles = virtual stages of the sampled tiles, tstride their stride)
  int dm = -1;               // QW dense pass: stage DMA issue, 0 at the barrier, 3 spread over
                             // the MFMA groups, -1 the default (score_qw.h SPREAD)
  int stagger = -1;          // QW dense pass at D = 384: 1 = waves 4-7 run their epilogue one
                             // stage late (score_qw.h STG), 0 = off, -1 = the default
};

// True when a kernel is instantiated for this row stride and query blocks per wave (1: 128
// queries per workgroup on 256-row tiles; 2: 256 queries on 128-row tiles).
bool qs_supported(int ld, int nq_blocks);
// Candidate buffer slots per query for k'.
int qs_cap(int kp);
// Launch on `st`; HCR_OK or an error code (hcr_last_error()).
int launch_qs(int dtype, const QsArgs& a, hipStream_t st);

constexpr int kQsRowTile = 256;       // row tile of the 1-block kernel (128 for 2 blocks)

// Wide query-stationary kernel (score_qw.h): 256 queries per workgroup held in VGPRs, full-K
// row stages; UNIT corpora without a row mask, ld = 384 or 768.
bool qw_supported(int ld);
int qw_rows(int ld, int nqb);         // rows per stage of the dense pass (the kernel's row tile)
int qw_sample_rows(int ld);           // ... of its MAXONLY pre-pass (256-row sampled tiles)
int qw_cap(int kp, int ld, int nqb);  // candidate buffer slots per query (0: k' too large)
int launch_qw(int dtype, const QsArgs& a, hipStream_t st);
constexpr int kQwQueries = 256;       // queries per QW workgroup (= QW_QT)
constexpr int kQwStages = 3;          // QW ring stages (= QW_NST)

// One-wave-per-SIMD query-stationary kernel (score_qw1.h): D = 1024, 192 queries per workgroup,
// UNIT corpora without a row mask.
bool qw1_supported(int ld);
int qw1_rows(int ld);                 // rows per stage (the kernel's row tile)
int qw1_queries(int ld);              // queries per workgroup
int qw1_cap(int kp, int ld);          // candidate buffer slots per query (0: k' too large)
int launch_qw1(int dtype, const QsArgs& a, hipStream_t st);
