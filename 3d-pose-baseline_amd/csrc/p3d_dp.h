// p3d_dp.h -- the data-parallel training step with its gradient all-reduce issued by this library
// (host code; included at the end of p3d.hip, after the model and its helpers).
//
// pure data parallelism -- every rank differentiates its own batch of 64, the flat fp32
// gradient (17.17 MB at cfg2) is averaged over the replicas, every rank applies the identical TF1
// Adam update (src/linear_model.py:137-145: one optimizer step per global batch).
//
// Why the library issues the collective itself (round 4): the step runs as ONE captured HIP graph
// (forward, backward, bucketed all-reduce, optimizer).  Issued through torch.distributed, every
// collective also leaves a torch Work whose end event the ProcessGroupNCCL watchdog thread polls;
// ROCm's hipEventQuery refuses an event whose stream is being captured (hipErrorCapturedEvent), so
// a Work of the eager warm-up steps still unreaped when the NCCL stream joined the capture killed
// the process from the watchdog thread (BENCH_r03: rc 134).  Here the step holds no torch object:
// librccl is called directly on a stream the library owns, from a communicator built from a unique
// id the ranks exchanged once over torch.distributed (p3d_comm_unique_id / p3d_comm_create).
//
// librccl is resolved at run time (dlopen + dlsym) from the library the process already uses --
// torch's copy, whose path the Python host passes -- so there is ONE RCCL in the process and
// libp3d.so gains no link-time dependency (CPU-only hosts load it, tests/test_abi_host.py).
//
// The step (p3d_train_step_dp), buckets as planned by p3d_grad_buckets (backward order):
//   compute stream: forward, output dgrad, ..., [bucket k's k_wgrad_multi, event g_k], ..., last dgrad
//   comm stream:    wait g_k -> all-reduce of bucket k's flat range -> event r_k     (k = 0, 1, ...)
//   compute stream: wait r_k -> TF1 Adam + re-pack of bucket k (the last one advances the step state)
// so bucket k's all-reduce overlaps the data gradients of the layers below it, while every
// optimizer launch stays on the compute queue (round 3 measured a comm-queue optimizer slowing
// every neighbouring dgrad launch: 155 vs 107 us per step at one rank; P3D_DP_ADAM=2 keeps that
// form).  One rank: the reduction is the identity (the mean of one replica), so the step issues no
// collective and forks no comm stream -- the same launches in the same order otherwise; N > 1: ncclAvg (RCCL pre-multiplies each contribution by
// 1/N; for N a power of two exactly the sum / N the host-staged gloo path computes).
#pragma once
#include <dlfcn.h>
#include <rccl/rccl.h>

struct p3d_comm {
  ncclComm_t nc = nullptr;
  int nranks = 0, rank = 0;
};

namespace {

struct RcclApi {
  void* h = nullptr;
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) err_str = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
};
RcclApi g_rccl;
std::mutex g_rccl_mu;

int rccl_fail(const char* what, ncclResult_t r) {
  return fail(P3D_ERR_HIP, std::string(what) + ": " + (g_rccl.err_str ? g_rccl.err_str(r) : "RCCL error") +
                               " (" + std::to_string((int)r) + ")");
}

int rccl_ready() {
  if (!g_rccl.h) return fail(P3D_ERR_STATE, "RCCL not loaded (p3d_comm_load)");
  return P3D_OK;
}

// flat [begin, end) of gradient bucket k (layers lowest[k] .. the previous bucket's lowest - 1)
void bucket_range(const p3d_model* m, int k, int64_t& fb, int64_t& fe) {
  const int nl = (int)m->layers.size();
  const int hi = k == 0 ? nl - 1 : m->bucket_lo[k - 1] - 1, lo = m->bucket_lo[k];
  fb = m->layers[lo].w;
  fe = hi + 1 < nl ? m->layers[hi + 1].w : m->n_flat;
}

// the N > 1 form: several ranks, or one forced into it (P3D_DP_FORCE_MULTI)
bool dp_multi(const p3d_model* m) { return m->comm->nranks > 1 || m->dp_force_multi; }

int dp_allreduce(p3d_model* m, float* buf, int64_t n, hipStream_t st) {
  // in place; the identity on one rank (nothing enqueued), the replica mean otherwise (ncclAvg: on a
  // forced 1-rank group the mean of one replica, still the identity)
  const ncclRedOp_t op = dp_multi(m) ? ncclAvg : ncclSum;
  const ncclResult_t r = g_rccl.all_reduce(buf, buf, (size_t)n, ncclFloat32, op, m->comm->nc, st);
  return r == ncclSuccess ? P3D_OK : rccl_fail("p3d_train_step_dp: ncclAllReduce", r);
}

}  // namespace

extern "C" int p3d_comm_load(const char* librccl_path) {
  std::lock_guard<std::mutex> g(g_rccl_mu);
  if (g_rccl.h) return P3D_OK;
  const char* path = (librccl_path && *librccl_path) ? librccl_path : "librccl.so.1";
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return fail(P3D_ERR_NOTFOUND, std::string("p3d_comm_load: ") + dlerror());
  RcclApi a;
  a.h = h;
#define P3D_SYM(field, name)                                                                \
  a.field = reinterpret_cast<decltype(a.field)>(dlsym(h, #name));                            \
  if (!a.field) { dlclose(h); return fail(P3D_ERR_NOTFOUND, "p3d_comm_load: " #name " missing in " + std::string(path)); }
  P3D_SYM(get_id, ncclGetUniqueId)
  P3D_SYM(init_rank, ncclCommInitRank)
  P3D_SYM(all_reduce, ncclAllReduce)
  P3D_SYM(destroy, ncclCommDestroy)
  P3D_SYM(err_str, ncclGetErrorString)
  P3D_SYM(group_start, ncclGroupStart)
  P3D_SYM(group_end, ncclGroupEnd)
#undef P3D_SYM
  g_rccl = a;
  return P3D_OK;
}

extern "C" int p3d_comm_unique_id(uint8_t* id, int64_t id_len) {
  if (!id || id_len < (int64_t)sizeof(ncclUniqueId)) return fail(P3D_ERR_ARG, "p3d_comm_unique_id: id needs 128 bytes");
  if (int rc = rccl_ready()) return rc;
  ncclUniqueId u;
  const ncclResult_t r = g_rccl.get_id(&u);
  if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
  memcpy(id, &u, sizeof(u));
  return P3D_OK;
}

extern "C" int p3d_comm_create(const uint8_t* id, int64_t id_len, int32_t nranks, int32_t rank, p3d_comm** out) {
  if (!id || !out || id_len < (int64_t)sizeof(ncclUniqueId)) return fail(P3D_ERR_ARG, "p3d_comm_create: null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(P3D_ERR_ARG, "p3d_comm_create: bad rank / size");
  if (int rc = rccl_ready()) return rc;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  p3d_comm* c = new p3d_comm();
  c->nranks = nranks;
  c->rank = rank;
  const ncclResult_t r = g_rccl.init_rank(&c->nc, nranks, u, rank);   // collective over the ranks
  if (r != ncclSuccess) {
    delete c;
    return rccl_fail("ncclCommInitRank", r);
  }
  *out = c;
  return P3D_OK;
}

extern "C" int p3d_comm_destroy(p3d_comm* c) {
  if (!c) return P3D_OK;
  if (c->nc && g_rccl.destroy) {
    const ncclResult_t r = g_rccl.destroy(c->nc);
    delete c;
    if (r != ncclSuccess) return rccl_fail("ncclCommDestroy", r);
    return P3D_OK;
  }
  delete c;
  return P3D_OK;
}

extern "C" int p3d_comm_allreduce(p3d_comm* c, void* buf, int64_t n, int32_t dtype, int32_t op, void* stream) {
  if (!c || (!buf && n > 0) || n < 0) return fail(P3D_ERR_ARG, "p3d_comm_allreduce: bad argument");
  if (dtype != P3D_DTYPE_F32 && dtype != P3D_DTYPE_F64) return fail(P3D_ERR_ARG, "p3d_comm_allreduce: f32 or f64");
  if (op < 0 || op > 2) return fail(P3D_ERR_ARG, "p3d_comm_allreduce: op 0 sum, 1 mean, 2 max");
  if (int rc = rccl_ready()) return rc;
  const ncclRedOp_t o = op == 0 ? ncclSum : op == 2 ? ncclMax : (c->nranks == 1 ? ncclSum : ncclAvg);
  const ncclResult_t r = g_rccl.all_reduce(buf, buf, (size_t)n, dtype == P3D_DTYPE_F32 ? ncclFloat32 : ncclFloat64,
                                           o, c->nc, (hipStream_t)stream);
  return r == ncclSuccess ? P3D_OK : rccl_fail("p3d_comm_allreduce: ncclAllReduce", r);
}

extern "C" int p3d_dp_attach(p3d_model* m, p3d_comm* c) {
  if (!m) return fail(P3D_ERR_ARG, "p3d_dp_attach: null model");
  m->comm = c;
  if (c && !m->cst) HIP_TRY(hipStreamCreateWithFlags(&m->cst, hipStreamNonBlocking));
  if (c && !m->cjoin) HIP_TRY(hipEventCreateWithFlags(&m->cjoin, hipEventDisableTiming));
  return P3D_OK;
}

// One data-parallel training step: p3d_train_fwd_bwd_lr, the all-reduce of the flat gradient
// (per bucket on the library's comm stream when p3d_grad_buckets planned buckets, else one
// all-reduce on the caller's stream after the backward), TF1 Adam + re-pack, step advance.
// Graph-capturable as a whole: the comm stream joins a capture through the bucket events and is
// joined back before the call returns.
extern "C" int p3d_train_step_dp(p3d_model* m, const float* x, const float* t, int64_t B, float* y,
                                 float keep_prob, uint64_t seed, int64_t row_offset, float lr0, float decay_steps,
                                 float decay_rate, float* loss_dev, void* stream) {
  if (!m) return fail(P3D_ERR_ARG, "p3d_train_step_dp: null model");
  if (!m->comm) return fail(P3D_ERR_STATE, "p3d_train_step_dp: no communicator (p3d_dp_attach)");
  if (int rc = rccl_ready()) return rc;
  hipStream_t st = (hipStream_t)stream;
  int rc = p3d_train_fwd_bwd_lr(m, x, t, B, y, keep_prob, seed, row_offset, lr0, decay_steps, decay_rate,
                                loss_dev, stream);
  if (rc) return rc;
  const int nb = (int)m->gev.size();
  // the backward ran the bucketed form (one weight-gradient launch + event per bucket) exactly when
  // p3d_backward's condition held: buckets planned, no max-norm (its clip gradient needs every G)
  const bool bucketed = nb > 0 && !m->cfg.max_norm && m->wgrad_multi && (int)m->bucket_lo.size() == nb &&
                        (int)m->bat.size() == nb;
  if (!bucketed) {
    if (dp_multi(m) && (rc = dp_allreduce(m, m->flat[1], m->n_flat, st))) return rc;
    return p3d_adam_apply(m, stream);
  }
  if (!dp_multi(m)) {
    // one replica: the mean of the gradients is the gradient itself and RCCL enqueues nothing for
    // it, so no comm-stream branch either (a forked branch in a captured graph puts its edges on
    // another hardware queue and slowed every launch of the step by 0.4-0.7 us, r04 A/B): each
    // bucket's optimizer follows on the compute stream
    if (m->dp_adam == 0) return p3d_adam_apply(m, stream);
    for (int k = 0; k < nb; ++k)
      if ((rc = p3d_adam_apply_bucket(m, k, stream))) return rc;
    return P3D_OK;
  }
  if ((int)m->rev.size() != nb) {
    for (hipEvent_t e : m->rev) HIP_TRY(hipEventDestroy(e));
    m->rev.assign((size_t)nb, nullptr);
    for (hipEvent_t& e : m->rev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  for (int k = 0; k < nb; ++k) {
    int64_t fb, fe;
    bucket_range(m, k, fb, fe);
    HIP_TRY(hipStreamWaitEvent(m->cst, m->gev[k], 0));
    if ((rc = dp_allreduce(m, m->flat[1] + fb, fe - fb, m->cst))) return rc;
    if (m->dp_adam == 2) {                         // optimizer on the comm stream behind its bucket
      if ((rc = p3d_adam_apply_bucket(m, k, m->cst))) return rc;
    } else {
      HIP_TRY(hipEventRecord(m->rev[k], m->cst));
    }
  }
  if (m->dp_adam == 2) {
    HIP_TRY(hipEventRecord(m->cjoin, m->cst));
    HIP_TRY(hipStreamWaitEvent(st, m->cjoin, 0));
    return P3D_OK;
  }
  if (m->dp_adam == 0) {                           // one optimizer pass after the last bucket
    for (int k = 0; k < nb; ++k) HIP_TRY(hipStreamWaitEvent(st, m->rev[k], 0));
    return p3d_adam_apply(m, stream);
  }
  for (int k = 0; k < nb; ++k) {                   // per bucket, on the compute stream
    HIP_TRY(hipStreamWaitEvent(st, m->rev[k], 0));
    if ((rc = p3d_adam_apply_bucket(m, k, stream))) return rc;
  }
  return P3D_OK;
}
