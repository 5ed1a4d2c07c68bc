/*
 * hcrag.h — C ABI of libhcrag_hip.so, the MI355X-native embedding + vector-retrieval core
 * for HC-RAG's hot path.  Plain pointers and sizes only; no C++ exceptions
 * cross this boundary; every call returns an hcr_status (0 = OK, < 0 = error class) and
 * hcr_last_error() gives a thread-local message.
 *
 * The reference has no FFI: its callers bind Python-level interfaces that sit on
 * third-party CPU engines.  Each entry point below names the reference interface it
 * replaces (file:line in /root/reference) — the ctypes binding a maintainer adds is in
 * INTEGRATION.md.
 *
 * Ownership / threading:
 *   - host buffers are borrowed for the duration of the call only; the library owns all
 *     device memory and its stream; host-pointer calls are synchronous.
 *   - *_device calls take device pointers and a hipStream_t (as void*) and are
 *     asynchronous on that stream (inputs already resident in HBM).
 *   - a handle is not re-entrant; different handles may be used from different threads.
 */
#ifndef HCRAG_H_
#define HCRAG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  HCR_OK = 0,
  HCR_EINVAL = -1,   /* invalid argument (the reference raises ValueError here) */
  HCR_EHIP = -2,     /* HIP runtime error */
  HCR_ERCCL = -3,    /* RCCL error (multi-device index exchange) */
  HCR_ENOMEM = -4,   /* device allocation failed */
  HCR_EIO = -5,      /* file / format error (encoder weights, vocab) */
  HCR_EINTERNAL = -6 /* internal consistency check failed (e.g. a candidate key naming a row
                        outside the index): the call is abandoned, the handle stays usable */
} hcr_status;

typedef enum { HCR_F16 = 0, HCR_BF16 = 1, HCR_F32 = 2 } hcr_dtype;

typedef enum {
  HCR_SCORE_COSINE = 0,     /* raw cosine: experiments/main.py:841 */
  HCR_SCORE_UNIT = 1        /* (cos + 1) / 2: experiments/isRelevant.py:208 */
} hcr_score_mode;

typedef struct hcr_index hcr_index;

/* Last error message of the calling thread ("" if none). */
const char* hcr_last_error(void);
/* Library version string. */
const char* hcr_version(void);
/* Number of visible HIP devices (0 when no GPU); never fails. */
int hcr_device_count(void);

/* ---------------------------------------------------------------------------------------
 * Node-embedding index (brute-force cosine top-k).
 * Replaces the embedding matrix of experiments/main.py:762 (np.array of the pickled
 * embeddings) and LlamaIndex SimpleVectorStore's embedding dict (reached from
 * query_interface.py:200-204, graph_builder.py:161,493-498).
 * ------------------------------------------------------------------------------------- */

/* Create an empty index on HIP device `device` for `dim`-wide rows stored as `dtype`
 * (HCR_F16 / HCR_BF16 / HCR_F32).  `capacity_rows` pre-reserves storage (0 = grow). */
int hcr_index_create(int device, int dim, int dtype, int64_t capacity_rows, hcr_index** out);
int hcr_index_destroy(hcr_index* index);
/* Drop all rows and the row mask, keeping device storage for reuse. */
int hcr_index_reset(hcr_index* index);

/* Append `n` host rows (`rows_dtype`, row-major n x dim).  Row ids are insertion order.
 * `normalize` = 1 stores each row L2-normalised (computed in fp64) before rounding to the
 * storage dtype; 0 stores the values as given (rounded).  Cosine is scale-invariant, so
 * either way the index ranks by sklearn cosine of the STORED (decoded) values.
 * Replaces DynamicEmbeddingGenerator's list append (experiments/embedding_generator.py:127)
 * + the matrix build (experiments/main.py:762). */
int hcr_index_add(hcr_index* index, const void* rows, int64_t n, int rows_dtype, int normalize);
/* Same from device memory, asynchronous on `stream` (a hipStream_t; NULL = the legacy default
 * stream, ordered after the caller's work on it). */
int hcr_index_add_device(hcr_index* index, const void* d_rows, int64_t n, int rows_dtype,
                         int normalize, void* stream);

/* Global id of this index's row 0 (row-sharded indexes: shard offset).  Search results
 * report id_offset + local row.  Fixed once hcr_index_add_ids has been used (HCR_EINVAL on a
 * different value): rows then carry explicit ids, and plain adds after that get the ids
 * id_offset + row at the time of the add. */
int hcr_index_set_id_offset(hcr_index* index, int64_t id_offset);
/* hcr_index_add with an explicit global id per row (host int64[n]); searches report these
 * ids for the appended rows (earlier rows keep id_offset + row).  Used by the multi-device
 * index's shards and by stores whose ids are not insertion order. */
int hcr_index_add_ids(hcr_index* index, const void* rows, int64_t n, int rows_dtype,
                      int normalize, const int64_t* ids);

int64_t hcr_index_size(const hcr_index* index);
int hcr_index_dim(const hcr_index* index);
int hcr_index_dtype(const hcr_index* index);

/* Copy stored rows [row0, row0+n) back to host as float32 (decoded storage values). */
int hcr_index_get_rows(const hcr_index* index, int64_t row0, int64_t n, float* out_rows);

/* Restrict searches to rows whose mask byte is non-zero (NULL clears the mask).  `n` must
 * equal the index size; rows appended later are visible until the mask is set again.
 * Replaces the category filter of experiments/main.py:872-885. */
int hcr_index_set_rowmask(hcr_index* index, const uint8_t* mask, int64_t n);

/* Batched top-k search: for each of `nq` float32 queries, the k rows of best cosine
 * (sklearn semantics in fp64 on the stored values; tie rule score desc, id asc), mapped
 * by `score_mode`, then kept only if score >= `threshold` (fp64; pass -INFINITY for none).
 * Outputs (host, nq x k): scores (float64, the exact fp64 cosine), ids (int64, -1 = empty
 * slot, score -inf).  Always the exact top-k: certified candidates (k <= 256) or, for the
 * queries the certificate cannot settle and for k > 256, an exact fp64 scan of every row.
 * Replaces cosine_similarity + np.argsort(...)[::-1][:top_k] + threshold filter of
 * experiments/main.py:841-849 (and :886-889), and get_top_k_embeddings behind
 * VectorContextRetriever (query_interface.py:200-204).  Any k >= 1: above 2048 every row's
 * exact key is sorted per query (query groups of <= 4 GiB of keys; corpora of < 2^31 rows). */
int hcr_search(hcr_index* index, const float* queries, int64_t nq, int k, int score_mode,
               double threshold, double* out_scores, int64_t* out_ids);

/* Device variant: queries (float32, nq x dim), outputs in device memory; fp64 scores so
 * that row-sharded results merge exactly across GPUs.  Kernels run on `stream` (NULL = the
 * legacy default stream); the call waits once per pass for the certificate count (DESIGN.md
 * §4) -- by default for the pass's last launch to store it in pinned host memory, which it does
 * after every write of the outputs (HCR_OPT_FLAG_READ) -- so outputs are final when it returns
 * and later work on `stream` is ordered after them. */
int hcr_search_device(hcr_index* index, const float* d_queries, int64_t nq, int k,
                      int score_mode, double threshold, double* d_out_scores,
                      int64_t* d_out_ids, void* stream);

/* Global seed across row shards (one index per shard: ranks of hcrag_amd.distributed or the
 * shards of one process).  Replaces nothing in the reference (it has one corpus):
 * it is the multi-GPU form of hcr_search_device's sampling seed, so that every shard appends
 * only the rows above a seed drawn from the WHOLE corpus' sample instead of its own.
 *   1. hcr_search_sample_device on every shard: its sampling pre-pass, the unit maxima copied to
 *      d_umax as [units][nq] floats (umax_cap floats available), its sampled row count.  units =
 *      0: this shard's route has no such sample -- search every shard with hcr_search_device.
 *   2. the caller gathers every shard's maxima ([sum of units][nq]; pad a shard's missing units
 *      with -INFINITY) and the sampled fraction (sum of sampled rows / sum of shard rows).
 *   3. hcr_search_seeded_device on every shard: the dense pass from that seed; outputs the
 *      shard's exact top k among the rows above the seed (fewer when fewer pass: score -inf, id
 *      -1) and d_out_bound[q] (fp64): every row of the shard outside its output scores <= it
 *      (exact cosine; -inf: none was left out).
 *   4. merge the shards' lists (hcr_merge_topk_device): a query's merged list is the exact top
 *      k where its k-th score is > every shard's bound; re-run the others with
 *      hcr_search_device on every shard.
 * Cosine scores, no threshold (score_mode COSINE, -INFINITY); 1 <= nq <= 16384, 1 <= k <= 256.
 * hcr_index_last_stats after step 3 covers steps 1 and 3 (the seeded call adds to them).  Step 3
 * right after step 1 on the same index and the same d_queries pointer reuses step 1's query
 * preparation, unless the index changed in between (add, reset, truncate, row mask, options other
 * than HCR_OPT_SAMPLE_STRIDE: the prep is then redone).  The CONTENTS of d_queries must not change
 * between the two calls: the reuse keys on the pointer and nq, not on the values.
 * Gathered units (step 3's `units`) up to 16384; above 4096 the seed select sorts them in LDS. */
int hcr_search_sample_device(hcr_index* index, const float* d_queries, int64_t nq, int k,
                             float* d_umax, int64_t umax_cap, int* units, int64_t* sampled_rows,
                             void* stream);
int hcr_search_seeded_device(hcr_index* index, const float* d_queries, int64_t nq, int k,
                             const float* d_umax_all, int units, double sampled_fraction,
                             double* d_out_scores, int64_t* d_out_ids, double* d_out_bound,
                             void* stream);

/* Exact fp64 cosine of every (query, row) pair, host outputs nq x size (float64).
 * Replaces the full-score vector of experiments/isRelevant.py:206 (batch_semantic_similarity
 * returns every node's score, in node order).  Intended for small indexes. */
int hcr_score_all(hcr_index* index, const float* queries, int64_t nq, int score_mode,
                  double* out_scores);

/* Statistics of the last search on this handle: candidates kept per query (k'), queries
 * whose top-k needed a widened candidate set, queries returned uncertified (always 0: the
 * exact fallback settles them), queries answered by the exact fallback scan and its rounds. */
typedef struct {
  int32_t kprime;
  int32_t widened_queries;
  int32_t uncertified_queries;
  int32_t partitions;
  int32_t score_launches;     /* score kernel launches timed (timing enabled only) */
  int32_t workgroups;         /* score kernel grid size of the first pass */
  double score_kernel_ms;     /* summed HIP-event time of those launches */
  int32_t unit_kernel;        /* 1: the UNIT score kernel ran (L2-normalised corpus, raw dot
                                 product as coarse score, widened certificate bound) */
  int32_t fallback_queries;   /* queries answered by the exact fp64 scan (K6/K7) */
  int32_t fallback_rounds;    /* K6/K7 rounds run (threshold tightenings + 1 per group; + the
                                 MFMA prefilter's round-0 histogram where it ran) */
  int32_t score_kernel;       /* dense score kernel of the first pass: 1 register-staged
                                 128 x 128 (fp32 rows), 3 v3 (256 x 16 / 256 x 64), 4 v4
                                 (256 x 256), 5 query-stationary QS, 6 wide query-stationary QW,
                                 7 QW1 (D = 1024: one wave per SIMD, 48 queries per wave) */
} hcr_search_stats;
int hcr_index_last_stats(const hcr_index* index, hcr_search_stats* out);
/* Enable (1) / disable (0) HIP-event timing of the fused score kernel (K2) on the stream it
 * is launched on; results appear in hcr_search_stats. */
int hcr_index_set_timing(hcr_index* index, int enable);

/* Tuning options of one index (results never change, only which exact kernel computes them).
 *   HCR_OPT_QW1: the large-batch kernel at D = 1024 (from 257 queries).  -1 / 1 = QW1 (the
 *                default), 0 = never QW1 (v4).  No effect at other dimensions.
 *   HCR_OPT_SAMPLE_STRIDE: the sampling pre-pass reads every value-th row tile (0 = the
 *                heuristic: the largest power of two in [16, 128] leaving >= 150 sampled 256-row
 *                tiles; 2 .. 4096 otherwise).  A denser sample
 *                gives a tighter seed (fewer candidate appends in the dense pass) at the cost of
 *                a longer pre-pass.
 *   HCR_OPT_QS_FORM: the query-stationary kernel's ring stages for 129-256 queries at D = 384:
 *                0 = the heuristic (= 3), 1 = 64-deep stages, 3 = 128-deep stages.
 *   HCR_OPT_PREPASS: the sampling pre-pass kernel: 0 = the heuristic (QW's form under a QW
 *                dense pass of several 256-query blocks, else v4's), 1 = the 256 x 256 v4
 *                kernel's MAXONLY form, 2 = QW's MAXONLY form (also under the QS dense pass, on
 *                an L2-normalised corpus without a row mask).
 *   HCR_OPT_QW_DM: how the wide query-stationary kernel (QW) issues a row stage's LDS-DMA:
 *                -1 = the default (3 with one 256-query block, else 0), 0 = right after the
 *                stage barrier, 3 = spread over the MFMA groups.  (1, 2, 4, 5: measured in r05,
 *                removed.)
 *   HCR_OPT_QW_MIN: the smallest batch the QW kernel takes (0 = the heuristic: 129).
 *   HCR_OPT_QW_STAGGER: QW at D = 384 -- waves 4-7 run each stage's top-k' test one stage
 *                late (beside the other waves' MFMAs): 1 = with two accumulator sets, 2 = with
 *                one, 0 = off, -1 = the default (2).
 *   HCR_OPT_FLAG_READ: how a search pass reads its certificate count back (its one host read):
 *                1 = a copy into pageable memory + stream synchronisation, 2 = a copy into
 *                pinned memory + synchronisation, 3 = a one-thread kernel stores it into pinned
 *                coherent host memory with a sequence number the host polls, then synchronises,
 *                4 = the same without the synchronisation; 0 = the default. */
typedef enum { HCR_OPT_QW1 = 1, HCR_OPT_SAMPLE_STRIDE = 3, HCR_OPT_QS_FORM = 4,
               HCR_OPT_PREPASS = 5, HCR_OPT_QW_DM = 6, HCR_OPT_QW_MIN = 7,
               HCR_OPT_QW_STAGGER = 8, HCR_OPT_FLAG_READ = 9 } hcr_index_option;
               /* (2: removed in 0.3) */
int hcr_index_set_option(hcr_index* index, int option, int value);

/* Test hooks (tests/test_exact_gpu.py; never set in production): per handle, off by default.
 *   HCR_TEST_PLANT_BAD_KEY: value 1 makes every later search on this handle plant a candidate
 *                key naming a row outside the index (as a defective score kernel could): the
 *                search must fail with HCR_EINTERNAL instead of gathering that row. */
typedef enum { HCR_TEST_PLANT_BAD_KEY = 1 } hcr_test_hook;
int hcr_index_test_hook(hcr_index* index, int hook, int value);

/* Merge g row-shards' per-query top-k lists (device, each [g][nq][k] scores fp64 + ids)
 * into the global top-k (score desc, id asc).  Used after the cross-GPU exchange of
 * SURVEY.md §8(e).  Asynchronous on `stream` for g x k <= 8192; deeper merges (one bitonic
 * sort of the (score, id) keys per query, deep_sort.hip) synchronise `stream` before
 * returning. */
int hcr_merge_topk_device(const double* d_scores, const int64_t* d_ids, int g, int64_t nq,
                          int k, double* d_out_scores, int64_t* d_out_ids, void* stream);

/* ---------------------------------------------------------------------------------------
 * Single-process multi-device index (one process drives all g devices).
 * Rows are sharded in contiguous blocks over `n_dev` devices (dev_ids may repeat: several
 * shards on one GPU); each hcr_multi_add splits its rows into n_dev blocks, ids stay insertion
 * order.  hcr_multi_search runs every shard's exact top-k concurrently (one host thread and
 * stream per shard), gathers the per-shard lists on dev_ids[0] -- RCCL sends to it over the
 * distinct devices (ncclCommInitAll), or peer copies when devices repeat, RCCL is absent or
 * its communicators cannot be created -- and merges them there (K5).  Same results as one hcr_index over all rows.  Replaces the
 * single matrix of experiments/main.py:762 / the vector store behind
 * query_interface.py:200-204 when the corpus spans the GPUs of a node.
 * ------------------------------------------------------------------------------------- */
typedef struct hcr_multi_index hcr_multi_index;
int hcr_multi_create(int n_dev, const int* dev_ids, int dim, int dtype, int64_t capacity_rows,
                     hcr_multi_index** out);
int hcr_multi_destroy(hcr_multi_index* m);
/* All or nothing: on failure no row of the call is added (shards that took their block drop it). */
int hcr_multi_add(hcr_multi_index* m, const void* rows, int64_t n, int rows_dtype, int normalize);
int hcr_multi_set_rowmask(hcr_multi_index* m, const uint8_t* mask, int64_t n);
int hcr_multi_search(hcr_multi_index* m, const float* queries, int64_t nq, int k, int score_mode,
                     double threshold, double* out_scores, int64_t* out_ids);
int64_t hcr_multi_size(const hcr_multi_index* m);
int hcr_multi_num_shards(const hcr_multi_index* m);
int64_t hcr_multi_shard_size(const hcr_multi_index* m, int shard);
/* 1: the last search gathered lists by RCCL point-to-point sends, 0: by peer copies. */
int hcr_multi_exchange_kind(const hcr_multi_index* m);
int hcr_multi_last_stats(const hcr_multi_index* m, hcr_search_stats* out);

/* ---------------------------------------------------------------------------------------
 * WordPiece tokenizer (host).  Replaces HF tokenizers 0.21.1 (Rust) BertNormalizer +
 * BertPreTokenizer + WordPiece reached through SentenceTransformer.encode
 * (experiments/embedding_generator.py:124) / HuggingFaceEmbedding (graph_builder.py:147).
 * ------------------------------------------------------------------------------------- */
typedef struct hcr_tok hcr_tok;
/* vocab.txt (one token per line, id = line number).  strip_accents: 1/0, or -1 = follow
 * `lowercase` (BERT uncased default). */
int hcr_wordpiece_create(const char* vocab_path, int lowercase, int strip_accents, hcr_tok** out);
int hcr_wordpiece_create_from_buffer(const char* vocab_data, int64_t len, int lowercase,
                                     int strip_accents, hcr_tok** out);
int hcr_wordpiece_destroy(hcr_tok* tok);
int32_t hcr_wordpiece_vocab_size(const hcr_tok* tok);
/* Tokenise n UTF-8 strings (byte lengths in text_lens, or NULL for NUL-terminated): ids /
 * mask are n x max_len ([CLS] .. [SEP], truncated, [PAD] padded), lengths[i] = tokens
 * including the two specials. */
int hcr_tokenize(const hcr_tok* tok, const char* const* texts, const int64_t* text_lens,
                 int64_t n, int max_len, int32_t* ids, int32_t* mask, int32_t* lengths);

/* ---------------------------------------------------------------------------------------
 * BERT sentence encoder.  Replaces SentenceTransformer('all-MiniLM-L6-v2').encode
 * (experiments/embedding_generator.py:21,124,197,337; experiments/main.py:807,869) and
 * HuggingFaceEmbedding(model_name=...)._get_text_embeddings (graph_builder.py:146-149,
 * query_interface.py:136-137): BertModel forward + Pooling(mean|cls) + Normalize.
 * ------------------------------------------------------------------------------------- */
typedef struct {
  int32_t vocab_size;      /* 30522 for all-MiniLM-L6-v2 */
  int32_t hidden;          /* 384; multiple of 64 */
  int32_t layers;          /* 6 */
  int32_t heads;           /* 12 */
  int32_t intermediate;    /* 1536; multiple of 64 */
  int32_t max_position;    /* 512 */
  int32_t type_vocab;      /* 2 */
  float layer_norm_eps;    /* 1e-12 */
  int32_t pooling;         /* 0 = mean over attention mask (sentence-transformers), 1 = CLS */
  int32_t normalize;       /* 1 = L2-normalise the pooled vector (Normalize module) */
} hcr_bert_config;
typedef struct hcr_encoder hcr_encoder;
/* compute_dtype:
 *   HCR_F32  reference precision (the reference encodes in fp32 torch,
 *            experiments/embedding_generator.py:124): projection GEMMs as three-term split-f16
 *            MFMA products (~22-bit operands, fp32 accumulation), fp32 attention/softmax/
 *            LayerNorm/residual; matches fp32 BertModel to ~1e-6.  The last partly filled
 *            round of a projection runs as K-chunks summed in chunk order, and which tiles
 *            fall in that round depends on the batch's packed token count: a sequence's bits
 *            are deterministic for a given batch but may differ by fp32 rounding (<= 1e-5)
 *            between batches that contain it (torch's own GEMMs are batch-dependent likewise);
 *   HCR_F16 / HCR_BF16  fast: f16 / bf16 MFMA operands (accumulation, LayerNorm, softmax and
 *            the residual stream fp32). */
int hcr_encoder_create(int device, const hcr_bert_config* cfg, int compute_dtype,
                       hcr_encoder** out);
int hcr_encoder_compute_dtype(const hcr_encoder* enc);
int hcr_encoder_destroy(hcr_encoder* enc);
/* HF BertModel state-dict tensor (fp32, row-major as stored).  Any prefix before
 * "embeddings." / "encoder." is ignored; pooler / head tensors are accepted and unused. */
int hcr_encoder_set_weight(hcr_encoder* enc, const char* name, const float* data, int64_t numel);
/* Upload all weights (checks every tensor of the config is present with the right size). */
int hcr_encoder_finalize(hcr_encoder* enc);
/* ids / mask: n x S int32 (token_type_ids are 0, as in SentenceTransformer.encode);
 * out: n x hidden fp32.  Synchronous, host buffers. */
int hcr_encode(hcr_encoder* enc, const int32_t* ids, const int32_t* mask, int64_t n, int S,
               float* out);
/* Same on device buffers, on `stream` (a hipStream_t; NULL = the legacy default stream).  Ids
 * must be in [0, vocab_size).  Only the tokens with mask 1 (plus position 0 under CLS pooling)
 * run through the layers: the packed token count is read back once per call, so the call waits
 * for the caller's earlier work on `stream` and for the packing kernel; the layers are then
 * enqueued asynchronously (batches of >= 128 sequences split over two internal streams that
 * `stream` waits for). */
int hcr_encode_device(hcr_encoder* enc, const int32_t* d_ids, const int32_t* d_mask, int64_t n,
                      int S, float* d_out, void* stream);

/* ---------------------------------------------------------------------------------------
 * Fused non-LLM isRelevant combiners.  Replaces the per-node Python
 * loops of experiments/isRelevant.py batch_entity_match (:300-324), batch_node_type_priority
 * (:327-346) and batch_isRelevant's combiners (:445-501) for nq queries x nn nodes each:
 *   semantic = (cos + 1) / 2 of cos_scores[q][j] (e.g. the exact top-k scores of hcr_search),
 *   entity   = |Q & N| / |Q| over entity bitsets (`words` u32 per set), 0.5 / 0.1 when the
 *              query has no entities (node has none / has some),
 *   type     = priority[intent[q]][node_type[node]] (a [n_intents][n_types] table; the
 *              caller maps unlisted types to the "unknown" column),
 *   llm      = llm_scores[q][j] (NULL = 0; the reference's LLM judge is out of scope),
 * combined per scorer (weights4 = semantic, llm, entity, type; NULL = the reference
 * defaults 0.3 / 0.45 / 0.15 / 0.10).  node_ids[q][j] picks the node (NULL: node j; < 0: a
 * padded slot, output -inf).  fp64, same operation order as the reference.
 * ------------------------------------------------------------------------------------- */
typedef enum {
  HCR_REL_COMPOSITE = 0,
  HCR_REL_PARALLEL = 1,
  HCR_REL_ROUTER = 2,
  HCR_REL_ROUTER_ALL = 3,
  HCR_REL_ROUTER_TWO_SEM_LLM = 4,
  HCR_REL_ROUTER_TWO_ENT_TYPE = 5,
  HCR_REL_SINGLE_SEM = 6,
  HCR_REL_SINGLE_LLM = 7,
  HCR_REL_SINGLE_ENT = 8,
  HCR_REL_SINGLE_TYPE = 9
} hcr_rel_scorer;
/* Host buffers, synchronous; node arrays have n_nodes entries. */
int hcr_relevance_combine(int device, const double* cos_scores, const int64_t* node_ids,
                          int64_t nq, int nn, int64_t n_nodes, const uint32_t* node_entity_bits,
                          const int32_t* node_entity_count, int words,
                          const uint32_t* query_entity_bits, const int32_t* node_type,
                          const int32_t* query_intent, const double* priority, int n_intents,
                          int n_types, const double* llm_scores, int scorer_type,
                          const double* weights4, double* out);
/* Device buffers (weights4 host), asynchronous on `stream`; no range checks. */
int hcr_relevance_combine_device(const double* d_cos_scores, const int64_t* d_node_ids,
                                 int64_t nq, int nn, const uint32_t* d_node_entity_bits,
                                 const int32_t* d_node_entity_count, int words,
                                 const uint32_t* d_query_entity_bits, const int32_t* d_node_type,
                                 const int32_t* d_query_intent, const double* d_priority,
                                 int n_types, const double* d_llm_scores, int scorer_type,
                                 const double* weights4, double* d_out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HCRAG_H_ */
