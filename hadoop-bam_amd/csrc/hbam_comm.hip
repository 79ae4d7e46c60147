// hbam_comm.hip — the Sort plugin's exchange step over RCCL (xGMI), behind the C ABI.
//
// Replaces what moves records between the Sort job's tasks in the reference: the
// TotalOrderPartitioner over InputSampler split points and Hadoop's map -> reduce shuffle
// (cli/plugins/Sort.java:131-170; SURVEY.md §8(b) hbam_sort_multi_gpu, §8(e) steps 2-3).  One
// rank per GPU; every call below is collective over the communicator.
//   * split points: each rank's regular key samples (k_sample_keys) in one ncclAllGather, the
//     nranks-1 quantiles of their sorted union on the host — the rule hadoop_bam/sort.py's
//     choose_split_points applies, so the gloo and RCCL paths pick the same points;
//   * exchange: the partition bounds of the local sorted run (k_sort_bounds), the nranks x nranks
//     (records, bytes) matrix in one ncclAllGather, then ONE ncclGroupStart/End of per-peer
//     ncclSend/ncclRecv (keys, voffsets, block sizes, payload bytes): on xGMI every peer pair has
//     its own link, so the grouped point-to-point form uses all 7 links at once where a ring
//     would serialise them; then hbam_sort_received orders what arrived.
// RCCL is opened with dlopen on the first hbam_comm_init (a context that never sorts across
// GPUs does not load it; inside a PyTorch process the already-loaded librccl.so.1 is reused).
#include <dlfcn.h>
#include <mutex>

#include <rccl/rccl.h>

// largest single point-to-point transfer of the Sort exchange (bytes)
constexpr uint64_t XCHG_CHUNK = 1ull << 30;

namespace {

struct RcclApi {
  bool ok = false;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      api.err = std::string("dlopen(librccl.so.1) failed: ") + (e ? e : "?");
      return;
    }
    bool all = true;
    auto sym = [&](const char* n) {
      void* p = dlsym(h, n);
      if (!p) {
        all = false;
        api.err += std::string(" missing ") + n;
      }
      return p;
    };
    api.GetUniqueId = (decltype(api.GetUniqueId))sym("ncclGetUniqueId");
    api.CommInitRank = (decltype(api.CommInitRank))sym("ncclCommInitRank");
    api.CommDestroy = (decltype(api.CommDestroy))sym("ncclCommDestroy");
    api.AllGather = (decltype(api.AllGather))sym("ncclAllGather");
    api.Send = (decltype(api.Send))sym("ncclSend");
    api.Recv = (decltype(api.Recv))sym("ncclRecv");
    api.GroupStart = (decltype(api.GroupStart))sym("ncclGroupStart");
    api.GroupEnd = (decltype(api.GroupEnd))sym("ncclGroupEnd");
    api.GetErrorString = (decltype(api.GetErrorString))sym("ncclGetErrorString");
    api.ok = all;
  });
  return api;
}

}  // namespace

struct hbam_comm {
  hbam_ctx* c = nullptr;  // nullptr once the context is destroyed first (comm_detach)
  int device = 0;
  ncclComm_t comm = nullptr;
  int32_t nranks = 0, rank = 0;
  // plan of the last size query (hbam_sort_exchange with out->payload == NULL)
  bool planned = false;
  uint64_t plan_n = 0, plan_bytes = 0;
  const void* plan_key = nullptr;
  std::vector<int64_t> plan_sp;
  std::vector<uint64_t> rec_b, byte_b;  // this rank's partition bounds (nranks + 1)
  std::vector<uint64_t> cnt;            // [src][dst][records, bytes]
};

namespace {

#define NCCLCHK(ctx, x)                                                                          \
  do {                                                                                           \
    ncclResult_t r_ = (x);                                                                       \
    if (r_ != ncclSuccess)                                                                       \
      return set_err((ctx), HBAM_EDEVICE, "%s:%d %s: %s", __FILE__, __LINE__, #x,                \
                     rccl().GetErrorString ? rccl().GetErrorString(r_) : "rccl error");          \
  } while (0)

int comm_check(hbam_ctx* c, hbam_comm* m) {
  if (!c || !m) return HBAM_EINVAL;
  if (m->c != c) return set_err(c, HBAM_EINVAL, "the communicator belongs to another context");
  return HBAM_OK;
}

// Every ncclGroupStart is matched by one ncclGroupEnd, on the error paths too: a group left
// open would turn this thread's next RCCL call into part of it and hang the peers.
struct GroupGuard {
  bool open = false;
  ncclResult_t start() {
    const ncclResult_t r = rccl().GroupStart();
    open = r == ncclSuccess;
    return r;
  }
  ncclResult_t end() {
    open = false;
    return rccl().GroupEnd();
  }
  ~GroupGuard() {
    if (open) (void)rccl().GroupEnd();
  }
};

}  // namespace

void comm_detach(hbam_comm* m) { m->c = nullptr; }

extern "C" int hbam_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return HBAM_EINVAL;
  RcclApi& R = rccl();
  if (!R.ok) return HBAM_EDEVICE;
  ncclUniqueId id;
  if (R.GetUniqueId(&id) != ncclSuccess) return HBAM_EDEVICE;
  static_assert(sizeof(id) == HBAM_UNIQUE_ID_BYTES, "ncclUniqueId size");
  memcpy(id_out, &id, sizeof id);
  return HBAM_OK;
}

extern "C" int hbam_comm_init(hbam_ctx* c, const uint8_t* id, int32_t nranks, int32_t rank, hbam_comm** out) {
  if (!c || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return HBAM_EINVAL;
  *out = nullptr;
  RcclApi& R = rccl();
  if (!R.ok) return set_err(c, HBAM_EDEVICE, "RCCL unavailable: %s", R.err.c_str());
  HIPCHK(c, hipSetDevice(c->device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  hbam_comm* m = new hbam_comm();
  m->c = c;
  m->device = c->device;
  m->nranks = nranks;
  m->rank = rank;
  const ncclResult_t r = R.CommInitRank(&m->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete m;
    return set_err(c, HBAM_EDEVICE, "ncclCommInitRank(%d, %d): %s", nranks, rank, R.GetErrorString(r));
  }
  c->comms.push_back(m);
  *out = m;
  return HBAM_OK;
}

// Either order of destruction is safe: with the context still alive its stream is drained and the
// communicator unregistered; after hbam_destroy (which drained that stream) only the device is used.
extern "C" void hbam_comm_destroy(hbam_comm* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  if (m->c) {
    (void)hipStreamSynchronize(m->c->stream);
    auto& v = m->c->comms;
    v.erase(std::remove(v.begin(), v.end(), m), v.end());
  }
  if (m->comm) (void)rccl().CommDestroy(m->comm);
  delete m;
}

extern "C" int hbam_comm_split_points(hbam_ctx* c, hbam_comm* m, const hbam_sorted_run* run,
                                      uint32_t samples_per_rank, int64_t* split_points) {
  int rc;
  if ((rc = comm_check(c, m))) return rc;
  if (!run || samples_per_rank == 0 || (m->nranks > 1 && !split_points) || (run->n && !run->key))
    return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t P = (uint64_t)m->nranks, S = samples_per_rank;
  int64_t* buf;  // [S + 1] local, then [P][S + 1] gathered
  if ((rc = ensure(c, B_X_SAMP, (P + 1) * (S + 1), &buf))) return rc;
  int64_t* gath = buf + (S + 1);
  k_sample_keys<<<grid_for(S, RS_WG), RS_WG, 0, c->stream>>>(run->key, run->n, samples_per_rank, buf);
  HIPCHK(c, hipGetLastError());
  NCCLCHK(c, rccl().AllGather(buf, gath, (S + 1) * 8, ncclUint8, m->comm, c->stream));
  std::vector<int64_t> h(P * (S + 1));
  HIPCHK(c, copy_sync(c, h.data(), gath, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<int64_t> all;
  for (uint64_t r = 0; r < P; ++r) {
    const int64_t k = h[r * (S + 1)];
    if (k < 0 || (uint64_t)k > S) return set_err(c, HBAM_EDEVICE, "rank %llu sent %lld samples", (unsigned long long)r, (long long)k);
    all.insert(all.end(), h.begin() + (long)(r * (S + 1) + 1), h.begin() + (long)(r * (S + 1) + 1 + (uint64_t)k));
  }
  std::sort(all.begin(), all.end());
  for (uint64_t j = 1; j < P; ++j)
    split_points[j - 1] = all.empty() ? 0 : all[(j * all.size()) / P];
  return HBAM_OK;
}

extern "C" int hbam_sort_exchange(hbam_ctx* c, hbam_comm* m, const hbam_sorted_run* run,
                                  const int64_t* split_points, hbam_sorted_run* out) {
  int rc;
  if ((rc = comm_check(c, m))) return rc;
  if (!run || !out || (m->nranks > 1 && !split_points)) return HBAM_EINVAL;
  if (run->n && (!run->key || !run->voffset || !run->block_size || !run->offsets || !run->payload))
    return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const uint32_t P = (uint32_t)m->nranks;
  const uint32_t me = (uint32_t)m->rank;
  RcclApi& R = rccl();
  if (!out->payload) {
    // ---- size query: partition + count all-gather
    m->rec_b.assign(P + 1, 0);
    m->byte_b.assign(P + 1, 0);
    if ((rc = hbam_sort_partition(c, run, split_points, P, m->rec_b.data(), m->byte_b.data()))) return rc;
    uint64_t* dcnt;
    if ((rc = ensure(c, B_X_CNT, 2ull * P * (P + 1), &dcnt))) return rc;
    std::vector<uint64_t> mine(2ull * P);
    for (uint32_t p = 0; p < P; ++p) {
      mine[2 * p] = m->rec_b[p + 1] - m->rec_b[p];
      mine[2 * p + 1] = m->byte_b[p + 1] - m->byte_b[p];
    }
    HIPCHK(c, hipMemcpyAsync(dcnt, mine.data(), 16ull * P, hipMemcpyHostToDevice, c->stream));
    NCCLCHK(c, R.AllGather(dcnt, dcnt + 2ull * P, 2ull * P, ncclUint64, m->comm, c->stream));
    m->cnt.assign(2ull * P * P, 0);
    HIPCHK(c, copy_sync(c, m->cnt.data(), dcnt + 2ull * P, 16ull * P * P, hipMemcpyDeviceToHost));
    uint64_t n = 0, bytes = 0;
    for (uint32_t s = 0; s < P; ++s) {
      n += m->cnt[(2ull * s * P) + 2ull * me];
      bytes += m->cnt[(2ull * s * P) + 2ull * me + 1];
    }
    m->planned = true;
    m->plan_n = run->n;
    m->plan_bytes = run->payload_bytes;
    m->plan_key = run->key;
    if (P > 1) m->plan_sp.assign(split_points, split_points + (P - 1));
    else m->plan_sp.clear();
    out->n = n;
    out->payload_bytes = bytes;
    return HBAM_OK;
  }
  // ---- the exchange proper: must follow the size query of the same run and split points
  if (!m->planned || m->plan_n != run->n || m->plan_bytes != run->payload_bytes || m->plan_key != run->key ||
      (P > 1 && !std::equal(m->plan_sp.begin(), m->plan_sp.end(), split_points)))
    return set_err(c, HBAM_EINVAL, "hbam_sort_exchange: call with out->payload == NULL first (same run, split points)");
  m->planned = false;
  uint64_t nr = 0, nb = 0;
  std::vector<uint64_t> roff(P + 1, 0), rboff(P + 1, 0);
  for (uint32_t s = 0; s < P; ++s) {
    roff[s + 1] = roff[s] + m->cnt[(2ull * s * P) + 2ull * me];
    rboff[s + 1] = rboff[s] + m->cnt[(2ull * s * P) + 2ull * me + 1];
  }
  nr = roff[P];
  nb = rboff[P];
  int64_t *rk, *rv;
  int32_t* rs;
  uint8_t* rp;
  if ((rc = ensure(c, B_X_KEY, nr + 1, &rk)) || (rc = ensure(c, B_X_VOFF, nr + 1, &rv)) ||
      (rc = ensure(c, B_X_BS, nr + 1, &rs)) || (rc = ensure(c, B_X_PAY, nb + 1, &rp)))
    return rc;
  HIPCHK(c, hipEventRecord(c->ev[12], c->stream));
  // every transfer goes out in pieces of at most XCHG_CHUNK bytes: a peer's payload at config
  // #5 is several GB, and no single point-to-point call above 2 GiB has been exercised; both sides
  // cut a (sender, receiver) pair's bytes at the same offsets, and RCCL matches the pieces in order
  auto send = [&](const void* ptr, uint64_t bytes, int peer) -> ncclResult_t {
    for (uint64_t o = 0; o < bytes; o += XCHG_CHUNK) {
      const ncclResult_t r = R.Send((const uint8_t*)ptr + o, std::min<uint64_t>(XCHG_CHUNK, bytes - o),
                                    ncclUint8, peer, m->comm, c->stream);
      if (r != ncclSuccess) return r;
    }
    return ncclSuccess;
  };
  auto recv = [&](void* ptr, uint64_t bytes, int peer) -> ncclResult_t {
    for (uint64_t o = 0; o < bytes; o += XCHG_CHUNK) {
      const ncclResult_t r = R.Recv((uint8_t*)ptr + o, std::min<uint64_t>(XCHG_CHUNK, bytes - o), ncclUint8,
                                    peer, m->comm, c->stream);
      if (r != ncclSuccess) return r;
    }
    return ncclSuccess;
  };
  GroupGuard group;
  NCCLCHK(c, group.start());
  for (uint32_t p = 0; p < P; ++p) {
    const uint64_t sr = m->rec_b[p + 1] - m->rec_b[p], sb = m->byte_b[p + 1] - m->byte_b[p];
    const uint64_t rr = roff[p + 1] - roff[p], rbb = rboff[p + 1] - rboff[p];
    const uint64_t r0 = m->rec_b[p], b0 = m->byte_b[p];
    if (sr) {
      NCCLCHK(c, send(run->key + r0, sr * 8, (int)p));
      NCCLCHK(c, send(run->voffset + r0, sr * 8, (int)p));
      NCCLCHK(c, send(run->block_size + r0, sr * 4, (int)p));
      NCCLCHK(c, send(run->payload + b0, sb, (int)p));
    }
    if (rr) {
      NCCLCHK(c, recv(rk + roff[p], rr * 8, (int)p));
      NCCLCHK(c, recv(rv + roff[p], rr * 8, (int)p));
      NCCLCHK(c, recv(rs + roff[p], rr * 4, (int)p));
      NCCLCHK(c, recv(rp + rboff[p], rbb, (int)p));
    }
  }
  NCCLCHK(c, group.end());
  HIPCHK(c, hipEventRecord(c->ev[13], c->stream));
  if ((rc = hbam_sort_received(c, rk, rv, rs, rp, nr, out))) return rc;
  c->timing.exchange_ms = ev_ms(c, 12, 13);  // (hbam_sort_received reset the rest)
  c->timing.comp_bytes = nb;
  return HBAM_OK;
}
