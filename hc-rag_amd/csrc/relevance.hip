// relevance.hip — fused non-LLM isRelevant combiners on the GPU.
//
// Restates experiments/isRelevant.py for every (query q, node j) pair of a batch:
//   semantic   = (cos + 1) / 2                                   (:197-210; cos is an input:
//                the exact fp64 cosine the search / score_all path already produced)
//   entity     = |set(Q) & set(N)| / |set(Q)|, and 0.5 / 0.1 when Q has no entities
//                (:300-324) -- the sets as bitsets over the batch's entity vocabulary
//   node type  = priority_matrix[intent][node_type], "unknown" column for unlisted types
//                (:128-169, :327-346) -- a [n_intents][n_types] table
//   llm        = an input score (the reference asks an LLM, :213-297: out of scope here)
// combined per ScorerType exactly as batch_isRelevant does (:445-501), in fp64 and in the
// reference's operation order, so equal inputs give bit-identical outputs.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hcrag.h"
#include "host_common.h"

namespace {

__global__ void relevance_kernel(const double* __restrict__ cos_s, const int64_t* __restrict__ ids,
                                 int64_t nq, int nn, const uint32_t* __restrict__ node_bits,
                                 const int32_t* __restrict__ node_nent, int words,
                                 const uint32_t* __restrict__ q_bits,
                                 const int32_t* __restrict__ node_type,
                                 const int32_t* __restrict__ q_intent,
                                 const double* __restrict__ prio, int n_types,
                                 const double* __restrict__ llm, int scorer, double w_sem,
                                 double w_llm, double w_ent, double w_type,
                                 double* __restrict__ out) {
  // no FMA contraction: every product / sum rounds separately, as in the Python reference
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq * (int64_t)nn) return;
  const int64_t q = i / nn;
  const int64_t id = ids ? ids[i] : (int64_t)(i - q * nn);
  if (id < 0) { out[i] = -INFINITY; return; }          // padded top-k slot
  const double sem = (cos_s[i] + 1.0) / 2.0;
  int qn = 0, inter = 0;
  for (int w = 0; w < words; ++w) {
    const uint32_t qb = q_bits[q * words + w];
    qn += __popc(qb);
    inter += __popc(qb & node_bits[id * words + w]);
  }
  const double ent = qn == 0 ? (node_nent[id] == 0 ? 0.5 : 0.1) : (double)inter / (double)qn;
  const double typ = prio[(int64_t)q_intent[q] * n_types + node_type[id]];
  const double l = llm ? llm[i] : 0.0;
  double s;
  switch (scorer) {
    case HCR_REL_PARALLEL: s = fmax(fmax(sem, l), fmax(ent, typ)); break;
    case HCR_REL_ROUTER: s = (sem + l + typ) / 3; break;
    case HCR_REL_ROUTER_ALL: s = (sem + l + ent + typ) / 4; break;
    case HCR_REL_ROUTER_TWO_SEM_LLM: s = (sem + l) / 2; break;
    case HCR_REL_ROUTER_TWO_ENT_TYPE: s = (ent + typ) / 2; break;
    case HCR_REL_SINGLE_SEM: s = sem; break;
    case HCR_REL_SINGLE_LLM: s = l; break;
    case HCR_REL_SINGLE_ENT: s = ent; break;
    case HCR_REL_SINGLE_TYPE: s = typ; break;
    default: s = sem * w_sem + l * w_llm + ent * w_ent + typ * w_type; break;   // COMPOSITE
  }
  out[i] = s;
}

template <typename T>
int upload(DevBuf& b, const T* src, size_t n, hipStream_t st) {
  CHECK(b.ensure(n * sizeof(T) + 16));
  if (n) HIPC(hipMemcpyAsync(b.p, src, n * sizeof(T), hipMemcpyHostToDevice, st));
  return HCR_OK;
}

}  // namespace

extern "C" int hcr_relevance_combine_device(
    const double* cos_scores, const int64_t* node_ids, int64_t nq, int nn,
    const uint32_t* node_entity_bits, const int32_t* node_entity_count, int words,
    const uint32_t* query_entity_bits, const int32_t* node_type, const int32_t* query_intent,
    const double* priority, int n_types, const double* llm_scores, int scorer_type,
    const double* weights4, double* out, void* stream) {
  if (nq < 0 || nn < 0 || words < 0 || n_types <= 0)
    return hcr_set_error(HCR_EINVAL, "relevance: bad sizes");
  if (nq == 0 || nn == 0) return HCR_OK;
  if (!cos_scores || !node_entity_count || !query_entity_bits || !node_type || !query_intent ||
      !priority || !out || (words > 0 && !node_entity_bits))
    return hcr_set_error(HCR_EINVAL, "relevance: NULL argument");
  if (scorer_type < HCR_REL_COMPOSITE || scorer_type > HCR_REL_SINGLE_TYPE)
    return hcr_set_errorf(HCR_EINVAL, "relevance: unknown scorer type %d", scorer_type);
  const double w0 = weights4 ? weights4[0] : 0.3, w1 = weights4 ? weights4[1] : 0.45;
  const double w2 = weights4 ? weights4[2] : 0.15, w3 = weights4 ? weights4[3] : 0.10;
  const int64_t tot = nq * (int64_t)nn;
  hipLaunchKernelGGL(relevance_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, cos_scores, node_ids, nq, nn, node_entity_bits,
                     node_entity_count, words, query_entity_bits, node_type, query_intent,
                     priority, n_types, llm_scores, scorer_type, w0, w1, w2, w3, out);
  HIPC(hipGetLastError());
  return HCR_OK;
}

extern "C" int hcr_relevance_combine(
    int device, const double* cos_scores, const int64_t* node_ids, int64_t nq, int nn,
    int64_t n_nodes, const uint32_t* node_entity_bits, const int32_t* node_entity_count,
    int words, const uint32_t* query_entity_bits, const int32_t* node_type,
    const int32_t* query_intent, const double* priority, int n_intents, int n_types,
    const double* llm_scores, int scorer_type, const double* weights4, double* out) {
  if (nq < 0 || nn < 0 || n_nodes < 0 || words < 0 || n_intents <= 0 || n_types <= 0)
    return hcr_set_error(HCR_EINVAL, "relevance: bad sizes");
  if (nq == 0 || nn == 0) return HCR_OK;
  if (!node_ids && (int64_t)nn > n_nodes)
    return hcr_set_error(HCR_EINVAL, "relevance: nn > n_nodes without node ids");
  for (int64_t q = 0; q < nq; ++q)
    if (query_intent[q] < 0 || query_intent[q] >= n_intents)
      return hcr_set_errorf(HCR_EINVAL, "relevance: query intent %d out of range", query_intent[q]);
  for (int64_t j = 0; j < n_nodes; ++j)
    if (node_type[j] < 0 || node_type[j] >= n_types)
      return hcr_set_errorf(HCR_EINVAL, "relevance: node type %d out of range", node_type[j]);
  if (node_ids)
    for (int64_t i = 0; i < nq * (int64_t)nn; ++i)
      if (node_ids[i] >= n_nodes) return hcr_set_error(HCR_EINVAL, "relevance: node id out of range");
  HIPC(hipSetDevice(device));
  hipStream_t st;
  HIPC(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  DevBuf dc, di, dnb, dne, dqb, dnt, dqi, dp, dl, dout;
  const size_t tot = (size_t)nq * nn;
  int rc = HCR_OK;
  do {
    if ((rc = upload(dc, cos_scores, tot, st))) break;
    if (node_ids && (rc = upload(di, node_ids, tot, st))) break;
    if ((rc = upload(dnb, node_entity_bits, (size_t)n_nodes * words, st))) break;
    if ((rc = upload(dne, node_entity_count, (size_t)n_nodes, st))) break;
    if ((rc = upload(dqb, query_entity_bits, (size_t)nq * words, st))) break;
    if ((rc = upload(dnt, node_type, (size_t)n_nodes, st))) break;
    if ((rc = upload(dqi, query_intent, (size_t)nq, st))) break;
    if ((rc = upload(dp, priority, (size_t)n_intents * n_types, st))) break;
    if (llm_scores && (rc = upload(dl, llm_scores, tot, st))) break;
    if ((rc = dout.ensure(tot * 8))) break;
    rc = hcr_relevance_combine_device(dc.as<double>(), node_ids ? di.as<int64_t>() : nullptr, nq, nn,
                                      dnb.as<uint32_t>(), dne.as<int32_t>(), words,
                                      dqb.as<uint32_t>(), dnt.as<int32_t>(), dqi.as<int32_t>(),
                                      dp.as<double>(), n_types,
                                      llm_scores ? dl.as<double>() : nullptr, scorer_type, weights4,
                                      dout.as<double>(), st);
    if (rc) break;
    hipError_t e = hipMemcpyAsync(out, dout.p, tot * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) rc = hcr_set_errorf(HCR_EHIP, "relevance: %s", hipGetErrorString(e));
  } while (0);
  (void)hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  for (DevBuf* b : {&dc, &di, &dnb, &dne, &dqb, &dnt, &dqi, &dp, &dl, &dout}) b->release();
  return rc;
}
