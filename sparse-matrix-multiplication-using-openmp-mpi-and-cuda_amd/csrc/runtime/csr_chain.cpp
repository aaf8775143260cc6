// `a4 --format mtx`: a chain of Matrix Market matrices on the CSR engine, in
// the native executable (the Python front-end's `apps/a4.py --format mtx` /
// models.spgemm.csr_chain, same input rules, same output bytes up to fp32
// summation order).  The reference's chain driver is
// sparse_matrix_mult.cu:402-681; its format is the folder of k x k uint64
// tiles, which `a4` keeps as the default.
//
//   mpiexec -n P a4 --format mtx <folder of *.mtx | A.mtx B.mtx ...> [--out C.mtx]
//
// Per rank (1D row-block, as the Python engine):
//   read      every rank parses 1/P of each file's text (libspmm_host
//             spmm_mtx_part / fill_part), the 1-rank rules applied at any P
//             (a file short of its header's nnz is rejected by every rank,
//             entries past it are ignored); entries go to their row owner
//             (MPI_Alltoallv), which builds its CSR row panel (sorted,
//             duplicates summed in fp32, symmetric storage expanded)
//   multiply  device-resident (GPU): each factor's row panel is uploaded once,
//             the right factor's panels are all-gathered device to device
//             (RCCL broadcasts over xGMI; --comm mpi stages through host MPI),
//             and the running product's row panel never leaves HBM between
//             products: csr_engine.cpp runs the bitmap-rank kernels for
//             uniform products and the binned LDS + long-row kernels for
//             skewed ones (R-MAT hubs), so no product falls back to the CPU.
//             --device cpu: the OpenMP Gustavson engine (libspmm_host).
//   write     C's panels go to rank 0 point to point, in rank order, and are
//             appended to the output as they arrive (spmm_mtx_write_*)
// stdout: "multiplying i i+1" per product (rank 0) and "time taken" per rank.
#include <dirent.h>
#include <mpi.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <iostream>
#include <numeric>
#include <regex>
#include <sstream>

#include "comm.hpp"
#include "csr_chain.hpp"
#include "csr_engine.hpp"
#include "rt.hpp"

extern "C" {
// libspmm_host.so
void* spmm_mtx_open(const char* path, int64_t* rows, int64_t* cols, int64_t* nnz, int* field, int* symmetry,
                    char* err, int errlen);
void spmm_mtx_close(void* handle);
int spmm_mtx_part(void* handle, int part, int nparts, int64_t* b0, int64_t* b1, int64_t* entries, int nthreads);
int64_t spmm_mtx_fill_part(void* handle, int64_t b0, int64_t b1, int64_t entries, int64_t* ri, int64_t* ci, double* v,
                           int nthreads);
void* spmm_mtx_write_begin(const char* path, int64_t m, int64_t n, int64_t nnz, int pattern);
int spmm_mtx_write_panel(void* handle, int64_t row0, int64_t mp, const int64_t* rp, const int32_t* ci, const float* v,
                         int nthreads);
int spmm_mtx_write_end(void* handle);
int64_t spmm_cpu_csr_spgemm_symbolic(int64_t m, int64_t n, const int64_t* Arp, const int32_t* Aci, const int64_t* Brp,
                                     const int32_t* Bci, int64_t* Crp, int nthreads);
int spmm_cpu_csr_spgemm_numeric(int64_t m, int64_t n, const int64_t* Arp, const int32_t* Aci, const float* Av,
                                const int64_t* Brp, const int32_t* Bci, const float* Bv, const int64_t* Crp,
                                int32_t* Cci, float* Cv, int nthreads);
}

namespace a4 {

namespace {

int64_t panel_lo(int64_t m, int p, int r) { return m * r / p; }   // parallel/partition.py row_panels

std::vector<std::string> mtx_paths(const std::vector<std::string>& inputs) {
  if (inputs.size() == 1) {
    if (DIR* d = opendir(inputs[0].c_str())) {
      std::vector<std::string> names;
      while (dirent* e = readdir(d)) {
        const std::string f = e->d_name;
        if (f.size() > 4 && f.compare(f.size() - 4, 4, ".mtx") == 0) names.push_back(f);
      }
      closedir(d);
      auto key = [](const std::string& f) {   // natural order: digit runs compare as numbers
        std::vector<std::pair<int64_t, std::string>> k;
        std::regex re("(\\d+)|(\\D+)");
        for (auto it = std::sregex_iterator(f.begin(), f.end(), re); it != std::sregex_iterator(); ++it)
          k.push_back((*it)[1].matched ? std::pair<int64_t, std::string>(std::stoll((*it)[1].str()), std::string())
                                       : std::pair<int64_t, std::string>(-1, (*it)[2].str()));
        return k;
      };
      std::sort(names.begin(), names.end(), [&](const std::string& a, const std::string& b) { return key(a) < key(b); });
      std::vector<std::string> out;
      for (auto& f : names) out.push_back(inputs[0] + "/" + f);
      return out;
    }
  }
  return inputs;
}

// This rank's row panel of a Matrix Market file (row_panels split).
Csr read_rowblock(const std::string& path, int rank, int world, int nthreads, int64_t* row0) {
  char err[512] = {0};
  int64_t m = 0, n = 0, nnz = 0;
  int field = 0, sym = 0;
  void* h = spmm_mtx_open(path.c_str(), &m, &n, &nnz, &field, &sym, err, sizeof err);
  A4_CHECK(h != nullptr, path + ": " + err);
  int64_t b0 = 0, b1 = 0, ne = 0;
  const bool whole = spmm_mtx_part(h, rank, world, &b0, &b1, &ne, nthreads) == 0;
  int64_t mine = whole ? ne : -1;
  std::vector<int64_t> counts(world);
  MPI_Allgather(&mine, 1, MPI_INT64_T, counts.data(), 1, MPI_INT64_T, MPI_COMM_WORLD);
  if (*std::min_element(counts.begin(), counts.end()) < 0) {
    spmm_mtx_close(h);
    throw Error(path + ": a part of the entry section does not hold whole entries");
  }
  const int64_t total = std::accumulate(counts.begin(), counts.end(), int64_t(0));
  if (total < nnz) {
    spmm_mtx_close(h);
    throw Error(path + ": file has " + std::to_string(total) + " entries, expected " + std::to_string(nnz));
  }
  const int64_t start = std::accumulate(counts.begin(), counts.begin() + rank, int64_t(0));
  const int64_t keep = std::max<int64_t>(0, std::min(counts[rank], nnz - start));   // entries past nnz: ignored
  std::vector<int64_t> ri(keep), cj(keep);
  std::vector<double> vv(keep, 1.0);
  if (keep) {
    const int per = field == 2 ? 2 : 3;
    const int64_t got = spmm_mtx_fill_part(h, b0, b1, keep, ri.data(), cj.data(), vv.data(), nthreads);
    if (got != counts[rank] * per) {
      spmm_mtx_close(h);
      throw Error(path + ": part " + std::to_string(rank) + " parsed " + std::to_string(got) + " tokens");
    }
  }
  spmm_mtx_close(h);
  for (int64_t e = 0; e < keep; ++e)
    A4_CHECK(ri[e] >= 0 && ri[e] < m && cj[e] >= 0 && cj[e] < n, path + ": coordinates out of range");
  if (sym == 1 || sym == 2 || sym == 3) {   // symmetric / skew / hermitian storage -> general
    const double sign = sym == 2 ? -1.0 : 1.0;
    const int64_t k0 = keep;
    for (int64_t e = 0; e < k0; ++e)
      if (ri[e] != cj[e]) {
        ri.push_back(cj[e]);
        cj.push_back(ri[e]);
        vv.push_back(sign * vv[e]);
      }
  }
  // entries to their row owners
  std::vector<int> dest(ri.size());
  std::vector<int64_t> scount(world, 0), rcount(world);
  for (size_t e = 0; e < ri.size(); ++e) {
    int r = (int)((ri[e] * world) / std::max<int64_t>(m, 1));   // first guess, then fix at panel edges
    while (r + 1 < world && ri[e] >= panel_lo(m, world, r + 1)) ++r;
    while (r > 0 && ri[e] < panel_lo(m, world, r)) --r;
    dest[e] = r;
    ++scount[r];
  }
  MPI_Alltoall(scount.data(), 1, MPI_INT64_T, rcount.data(), 1, MPI_INT64_T, MPI_COMM_WORLD);
  std::vector<int64_t> sdisp(world + 1, 0), rdisp(world + 1, 0);
  for (int r = 0; r < world; ++r) {
    sdisp[r + 1] = sdisp[r] + scount[r];
    rdisp[r + 1] = rdisp[r] + rcount[r];
  }
  A4_CHECK(sdisp[world] < (int64_t)INT32_MAX / 3 && rdisp[world] < (int64_t)INT32_MAX / 3,
           "a Matrix Market panel too large for one MPI exchange");
  std::vector<int64_t> sbuf(3 * sdisp[world]), fill(sdisp.begin(), sdisp.end() - 1);
  for (size_t e = 0; e < ri.size(); ++e) {
    const int64_t at = fill[dest[e]]++;
    sbuf[3 * at] = ri[e];
    sbuf[3 * at + 1] = cj[e];
    std::memcpy(&sbuf[3 * at + 2], &vv[e], 8);
  }
  std::vector<int64_t> rbuf(3 * rdisp[world]);
  std::vector<int> sc(world), sd(world), rc(world), rd(world);
  for (int r = 0; r < world; ++r) {
    sc[r] = (int)(3 * scount[r]);
    sd[r] = (int)(3 * sdisp[r]);
    rc[r] = (int)(3 * rcount[r]);
    rd[r] = (int)(3 * rdisp[r]);
  }
  MPI_Alltoallv(sbuf.data(), sc.data(), sd.data(), MPI_INT64_T, rbuf.data(), rc.data(), rd.data(), MPI_INT64_T,
                MPI_COMM_WORLD);
  // CSR of the panel: sort by (row, col), sum duplicates in fp32 (models/ops from_coo)
  const int64_t lo = panel_lo(m, world, rank), hi = rank == world - 1 ? m : panel_lo(m, world, rank + 1);
  const int64_t nr = rdisp[world];
  std::vector<int64_t> idx(nr);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
    return rbuf[3 * a] != rbuf[3 * b] ? rbuf[3 * a] < rbuf[3 * b] : rbuf[3 * a + 1] < rbuf[3 * b + 1];
  });
  Csr P;
  P.m = hi - lo;
  P.n = n;
  P.rp.assign(P.m + 1, 0);
  for (int64_t t = 0; t < nr; ++t) {
    const int64_t e = idx[t];
    double d;
    std::memcpy(&d, &rbuf[3 * e + 2], 8);
    const int64_t r = rbuf[3 * e] - lo;
    const int32_t c = (int32_t)rbuf[3 * e + 1];
    if (t > 0 && rbuf[3 * idx[t - 1]] == rbuf[3 * e] && rbuf[3 * idx[t - 1] + 1] == rbuf[3 * e + 1]) {
      P.v.back() += (float)d;
    } else {
      P.ci.push_back(c);
      P.v.push_back((float)d);
      ++P.rp[r + 1];
    }
  }
  for (int64_t r = 0; r < P.m; ++r) P.rp[r + 1] += P.rp[r];
  *row0 = lo;
  return P;
}

// Every rank's row panel of B, concatenated in rank order (MPI all-gather).
Csr allgather_rows(const Csr& panel, int world) {
  if (world == 1) return panel;
  const int64_t mine[2] = {panel.m, panel.nnz()};
  std::vector<int64_t> meta(2 * world);
  MPI_Allgather(mine, 2, MPI_INT64_T, meta.data(), 2, MPI_INT64_T, MPI_COMM_WORLD);
  std::vector<int> cm(world), dm(world), ce(world), de(world);
  int64_t M = 0, E = 0;
  for (int r = 0; r < world; ++r) {
    A4_CHECK(M + meta[2 * r] < INT32_MAX && E + meta[2 * r + 1] < INT32_MAX, "right factor too large for MPI");
    cm[r] = (int)meta[2 * r];
    dm[r] = (int)M;
    ce[r] = (int)meta[2 * r + 1];
    de[r] = (int)E;
    M += meta[2 * r];
    E += meta[2 * r + 1];
  }
  std::vector<int64_t> cnt(panel.m);
  for (int64_t i = 0; i < panel.m; ++i) cnt[i] = panel.rp[i + 1] - panel.rp[i];
  Csr B;
  B.m = M;
  B.n = panel.n;
  std::vector<int64_t> all(M);
  MPI_Allgatherv(cnt.data(), (int)panel.m, MPI_INT64_T, all.data(), cm.data(), dm.data(), MPI_INT64_T, MPI_COMM_WORLD);
  B.rp.assign(M + 1, 0);
  for (int64_t i = 0; i < M; ++i) B.rp[i + 1] = B.rp[i] + all[i];
  B.ci.resize(E);
  B.v.resize(E);
  MPI_Allgatherv(panel.ci.data(), (int)panel.nnz(), MPI_INT32_T, B.ci.data(), ce.data(), de.data(), MPI_INT32_T,
                 MPI_COMM_WORLD);
  MPI_Allgatherv(panel.v.data(), (int)panel.nnz(), MPI_FLOAT, B.v.data(), ce.data(), de.data(), MPI_FLOAT,
                 MPI_COMM_WORLD);
  return B;
}

Csr cpu_spgemm(const Csr& A, const Csr& B, int nthreads) {
  Csr C;
  C.m = A.m;
  C.n = B.n;
  C.rp.assign(A.m + 1, 0);
  const int64_t nnz = spmm_cpu_csr_spgemm_symbolic(A.m, B.n, A.rp.data(), A.ci.data(), B.rp.data(), B.ci.data(),
                                                   C.rp.data(), nthreads);
  C.ci.resize(nnz);
  C.v.resize(nnz);
  spmm_cpu_csr_spgemm_numeric(A.m, B.n, A.rp.data(), A.ci.data(), A.v.data(), B.rp.data(), B.ci.data(), B.v.data(),
                              C.rp.data(), C.ci.data(), C.v.data(), nthreads);
  return C;
}

// Every rank's device row panel of B, concatenated in rank order: the row
// counts through host MPI (small), columns and values device to device
// (Comm::allgatherv_dev: RCCL broadcasts over xGMI).
DCsr allgather_rows_dev(const DCsr& panel, Comm& comm, hipStream_t s) {
  const int world = comm.world();
  if (world == 1) {
    DCsr B;
    B.m = panel.m;
    B.n = panel.n;
    B.nnz = panel.nnz;
    B.rp = DevBuf<int64_t>(panel.m + 1, s);
    B.ci = DevBuf<int32_t>(std::max<int64_t>(panel.nnz, 1), s);
    B.v = DevBuf<float>(std::max<int64_t>(panel.nnz, 1), s);
    A4_HIP(hipMemcpyAsync(B.rp.get(), panel.rp.get(), (panel.m + 1) * 8, hipMemcpyDeviceToDevice, s));
    if (panel.nnz) {
      A4_HIP(hipMemcpyAsync(B.ci.get(), panel.ci.get(), panel.nnz * 4, hipMemcpyDeviceToDevice, s));
      A4_HIP(hipMemcpyAsync(B.v.get(), panel.v.get(), panel.nnz * 4, hipMemcpyDeviceToDevice, s));
    }
    return B;
  }
  const int64_t mine[2] = {panel.m, panel.nnz};
  std::vector<int64_t> meta(2 * world);
  MPI_Allgather(mine, 2, MPI_INT64_T, meta.data(), 2, MPI_INT64_T, MPI_COMM_WORLD);
  std::vector<int> cm(world), dm(world);
  int64_t M = 0, E = 0;
  std::vector<size_t> cb(world);
  for (int r = 0; r < world; ++r) {
    A4_CHECK(M + meta[2 * r] < INT32_MAX, "right factor has too many rows");
    cm[r] = (int)meta[2 * r];
    dm[r] = (int)M;
    M += meta[2 * r];
    cb[r] = (size_t)meta[2 * r + 1] * 4;
    E += meta[2 * r + 1];
  }
  std::vector<int64_t> rp_local(panel.m + 1);
  A4_HIP(hipMemcpyAsync(rp_local.data(), panel.rp.get(), (panel.m + 1) * 8, hipMemcpyDeviceToHost, s));
  A4_HIP(hipStreamSynchronize(s));
  std::vector<int64_t> cnt(panel.m), all(M);
  for (int64_t i = 0; i < panel.m; ++i) cnt[i] = rp_local[i + 1] - rp_local[i];
  MPI_Allgatherv(cnt.data(), (int)panel.m, MPI_INT64_T, all.data(), cm.data(), dm.data(), MPI_INT64_T, MPI_COMM_WORLD);
  std::vector<int64_t> rp(M + 1, 0);
  for (int64_t i = 0; i < M; ++i) rp[i + 1] = rp[i] + all[i];
  DCsr B;
  B.m = M;
  B.n = panel.n;
  B.nnz = E;
  B.rp = DevBuf<int64_t>(M + 1, s);
  A4_HIP(hipMemcpyAsync(B.rp.get(), rp.data(), (M + 1) * 8, hipMemcpyHostToDevice, s));
  B.ci = DevBuf<int32_t>(std::max<int64_t>(E, 1), s);
  B.v = DevBuf<float>(std::max<int64_t>(E, 1), s);
  comm.allgatherv_dev(panel.ci.get(), B.ci.get(), cb, s);
  comm.allgatherv_dev(panel.v.get(), B.v.get(), cb, s);
  return B;
}

// Point-to-point transfers in pieces of < 2^31 elements (MPI counts are int).
constexpr int64_t kMsg = int64_t(1) << 28;
template <typename T>
void send_big(const T* p, int64_t n, MPI_Datatype t, int dst, int tag) {
  for (int64_t o = 0; o < n; o += kMsg) MPI_Send(p + o, (int)std::min(kMsg, n - o), t, dst, tag, MPI_COMM_WORLD);
}
template <typename T>
void recv_big(T* p, int64_t n, MPI_Datatype t, int src, int tag) {
  for (int64_t o = 0; o < n; o += kMsg)
    MPI_Recv(p + o, (int)std::min(kMsg, n - o), t, src, tag, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
}

// Rows row0.. of C from every rank to rank 0, appended to the file in rank order.
void write_rows(const std::string& path, const Csr& P, int64_t row0, int rank, int world, int nthreads) {
  int64_t mine[2] = {P.m, P.nnz()}, tot[2] = {0, 0};
  MPI_Allreduce(mine, tot, 2, MPI_INT64_T, MPI_SUM, MPI_COMM_WORLD);
  if (rank != 0) {
    const int64_t hdr[3] = {row0, P.m, P.nnz()};
    MPI_Send(hdr, 3, MPI_INT64_T, 0, 10, MPI_COMM_WORLD);
    if (P.m) send_big(P.rp.data(), P.m + 1, MPI_INT64_T, 0, 11);
    if (P.nnz()) {
      send_big(P.ci.data(), P.nnz(), MPI_INT32_T, 0, 12);
      send_big(P.v.data(), P.nnz(), MPI_FLOAT, 0, 13);
    }
    return;
  }
  void* w = spmm_mtx_write_begin(path.c_str(), tot[0], P.n, tot[1], 0);
  A4_CHECK(w != nullptr, "cannot open " + path + " for writing");
  int rc = spmm_mtx_write_panel(w, row0, P.m, P.rp.data(), P.ci.data(), P.v.data(), nthreads);
  for (int r = 1; r < world && rc == 0; ++r) {
    int64_t hdr[3];
    MPI_Recv(hdr, 3, MPI_INT64_T, r, 10, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    Csr Q;
    Q.m = hdr[1];
    Q.rp.assign(Q.m + 1, 0);
    Q.ci.resize(hdr[2]);
    Q.v.resize(hdr[2]);
    if (Q.m) recv_big(Q.rp.data(), Q.m + 1, MPI_INT64_T, r, 11);
    if (hdr[2]) {
      recv_big(Q.ci.data(), hdr[2], MPI_INT32_T, r, 12);
      recv_big(Q.v.data(), hdr[2], MPI_FLOAT, r, 13);
    }
    rc = spmm_mtx_write_panel(w, hdr[0], Q.m, Q.rp.data(), Q.ci.data(), Q.v.data(), nthreads);
  }
  const int rc2 = spmm_mtx_write_end(w);
  A4_CHECK(rc == 0 && rc2 == 0, "writing " + path + " failed");
}

}  // namespace

int run_mtx(const MtxOptions& o, int rank, int world) {
  const std::vector<std::string> paths = mtx_paths(o.inputs);
  A4_CHECK(!paths.empty(), "no Matrix Market files");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  const bool gpu = o.device == "hip" || (o.device == "auto" && ndev > 0);
  A4_CHECK(!gpu || ndev > 0, "--device hip but no GPU is visible");
  hipStream_t s = nullptr;
  std::unique_ptr<Comm> comm;
  std::string comm_kind = "mpi";
  if (gpu) {
    A4_HIP(hipSetDevice(o.local_rank % ndev));
    A4_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    comm_kind = o.comm;
    if (comm_kind == "auto") {
      int local_size = world;
      if (const char* x = std::getenv("MPI_LOCALNRANKS")) local_size = std::atoi(x);
      comm_kind = (world > 1 && local_size <= ndev) ? "rccl" : "mpi";
    }
    comm = comm_kind == "rccl" ? make_rccl_comm(o.timeout) : make_mpi_comm();
  }
  int64_t row0 = 0, cpu_products = 0;
  int64_t flops = 0;
  EngineStats es;
  std::vector<double> t_products;   // device products: wall seconds each (upload / gather excluded)
  const double t0 = now_s();
  Csr P = read_rowblock(paths[0], rank, world, o.threads, &row0);
  DCsr Pd;
  if (gpu) Pd = dcsr_upload(P, s);   // the running product stays in HBM from here on
  for (size_t i = 1; i < paths.size(); ++i) {
    if (rank == 0 && !o.quiet) std::cout << "multiplying " << i << " " << i + 1 << std::endl;
    int64_t brow0 = 0;
    const Csr Bp = read_rowblock(paths[i], rank, world, o.threads, &brow0);
    if (gpu) {
      const DCsr Bpd = dcsr_upload(Bp, s);
      const DCsr B = allgather_rows_dev(Bpd, *comm, s);
      A4_CHECK(B.m == Pd.n, paths[i] + ": " + std::to_string(B.m) + " rows, the product so far has " +
                               std::to_string(Pd.n) + " columns");
      int64_t products = 0;
      A4_HIP(hipStreamSynchronize(s));   // per-product wall time: operands resident, C complete
      const double tp = now_s();
      DCsr C = dev_spgemm(Pd, B, s, &es, &products);
      A4_HIP(hipStreamSynchronize(s));
      t_products.push_back(now_s() - tp);
      flops += 2 * products;
      Pd = std::move(C);
    } else {
      const Csr B = allgather_rows(Bp, world);
      A4_CHECK(B.m == P.n, paths[i] + ": " + std::to_string(B.m) + " rows, the product so far has " +
                               std::to_string(P.n) + " columns");
      for (int64_t e = 0; e < P.nnz(); ++e) flops += 2 * (B.rp[P.ci[e] + 1] - B.rp[P.ci[e]]);
      P = cpu_spgemm(P, B, o.threads);
      ++cpu_products;
    }
  }
  if (gpu) P = dcsr_download(Pd, s);
  const double t1 = now_s();
  write_rows(o.out, P, row0, rank, world, o.threads);
  const double t2 = now_s();
  int64_t fl_all = 0;
  MPI_Reduce(&flops, &fl_all, 1, MPI_INT64_T, MPI_SUM, 0, MPI_COMM_WORLD);
  if (rank == 0 && !o.metrics.empty()) {
    std::ofstream m(o.metrics);
    m << "{\"engine\": \"native\", \"format\": \"mtx\", \"device\": \"" << (gpu ? "hip" : "cpu")
      << "\", \"device_resident\": " << (gpu ? "true" : "false") << ", \"comm\": \"" << comm_kind
      << "\", \"ranks\": " << world << ", \"n_files\": " << paths.size() << ", \"flops\": " << fl_all
      << ", \"gpu_products\": " << (es.bitmap + es.binned) << ", \"gpu_bitmap_products\": " << es.bitmap
      << ", \"gpu_binned_products\": " << es.binned << ", \"gpu_long_rows\": " << es.long_rows
      << ", \"host_resorted_rows\": " << es.resorted_rows << ", \"device_sorted_rows\": " << es.device_sorted_rows
      << ", \"cpu_products\": " << cpu_products << ", \"t_products_s\": [";
    for (size_t i = 0; i < t_products.size(); ++i) m << (i ? ", " : "") << t_products[i];
    m << "], \"t_chain_s\": " << (t1 - t0)
      << ", \"t_write_s\": " << (t2 - t1) << "}\n";
  }
  Pd = DCsr();
  comm.reset();
  if (s) (void)hipStreamDestroy(s);
  MPI_Barrier(MPI_COMM_WORLD);
  return 0;
}

}  // namespace a4
