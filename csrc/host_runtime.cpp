// Native host runtime pieces of the data pipeline (CPU side of an MI355X node).
//
// Reference: MTLabeledBGRImgToBatch (S/dataset/image/MTLabeledBGRImgToBatch.scala:26) assembles a batch with a
// thread per core, BGRImgCropper / HFlip / BGRImgNormalizer (S/dataset/image/*.scala) do the per-image work, and
// utils/ThreadPool.scala:130-164 (invokeAndWait / invokeAndWait2 with timeout) runs the tasks.
//
// Here one persistent std::thread pool (sized once; the GIL is released for the whole call) crops, flips,
// reorders BGR->RGB and normalises uint8 HWC images straight into a (pinned) fp32 NCHW batch, so a Python
// loader thread only hands over pointers. Work is split by image and by channel row blocks so a batch of a
// few large images still spreads over every worker.
#include <torch/extension.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>
#include <string>
#include <cstdlib>

namespace bigdl_host {

class ThreadPool {
 public:
  explicit ThreadPool(int n) : stop_(false) {
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return (int)workers_.size(); }
  // Runs fn(i) for i in [0, n) on the pool and the calling thread; returns when all are done.
  void parallel_for(int64_t n, const std::function<void(int64_t)>& fn) {
    if (n <= 0) return;
    std::atomic<int64_t> next(0), done(0);
    auto body = [&] {
      for (int64_t i; (i = next.fetch_add(1)) < n;) {
        fn(i);
        done.fetch_add(1);
      }
    };
    const int helpers = (int)std::min<int64_t>(n - 1, (int64_t)workers_.size());
    std::atomic<int> finished(0);
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int h = 0; h < helpers; ++h)
        tasks_.push_back([&] {
          body();
          finished.fetch_add(1);
        });
    }
    cv_.notify_all();
    body();
    while (finished.load() < helpers) std::this_thread::yield();
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> task;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [this] { return stop_ || !tasks_.empty(); });
        if (stop_ && tasks_.empty()) return;
        task = std::move(tasks_.back());
        tasks_.pop_back();
      }
      task();
    }
  }
  std::vector<std::thread> workers_;
  std::vector<std::function<void()>> tasks_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_;
};

// One process-wide pool; `want` threads in total (caller included), 0 = keep the current / hardware default.
ThreadPool& pool(int want) {
  static std::mutex m;
  static std::unique_ptr<ThreadPool> p;
  static int cur = 0;
  std::lock_guard<std::mutex> g(m);
  int n = want > 0 ? want : (cur > 0 ? cur : (int)std::max(1u, std::thread::hardware_concurrency()));
  if (n > 64) n = 64;
  if (!p || n != cur) {
    p.reset();
    p.reset(new ThreadPool(n - 1));
    cur = n;
  }
  return *p;
}

// images: list of uint8 [H_i, W_i, 3] (BGR, contiguous); params int32 [N, 3] = (y0, x0, flip);
// out fp32 [N, 3, OH, OW]; mean / std in output channel order (R,G,B if to_rgb) on the 0..255 scale.
void assemble_batch(const std::vector<torch::Tensor>& images, const torch::Tensor& params, const torch::Tensor& out,
                    std::vector<double> mean, std::vector<double> stdv, bool to_rgb, int64_t threads) {
  const int64_t N = (int64_t)images.size();
  TORCH_CHECK(out.dim() == 4 && out.size(0) == N && out.size(1) == 3 && out.scalar_type() == at::kFloat &&
                  out.is_contiguous() && !out.is_cuda(),
              "assemble_batch: out must be a contiguous CPU fp32 [N, 3, OH, OW] tensor");
  TORCH_CHECK(params.dim() == 2 && params.size(0) == N && params.size(1) == 3 && params.scalar_type() == at::kInt &&
                  params.is_contiguous(),
              "assemble_batch: params must be int32 [N, 3]");
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "assemble_batch: mean/std need 3 values");
  const int64_t OH = out.size(2), OW = out.size(3);
  std::vector<const uint8_t*> src(N);
  std::vector<int64_t> Hs(N), Ws(N);
  const int32_t* pr = params.data_ptr<int32_t>();
  for (int64_t i = 0; i < N; ++i) {
    const auto& im = images[i];
    TORCH_CHECK(im.dim() == 3 && im.size(2) == 3 && im.scalar_type() == at::kByte && im.is_contiguous() && !im.is_cuda(),
                "assemble_batch: image ", i, " must be contiguous CPU uint8 [H, W, 3]");
    Hs[i] = im.size(0);
    Ws[i] = im.size(1);
    TORCH_CHECK(pr[3 * i] >= 0 && pr[3 * i + 1] >= 0 && pr[3 * i] + OH <= Hs[i] && pr[3 * i + 1] + OW <= Ws[i],
                "assemble_batch: crop window of image ", i, " out of bounds");
    src[i] = im.data_ptr<uint8_t>();
  }
  float* dst = out.data_ptr<float>();
  float scale[3], shift[3];
  for (int c = 0; c < 3; ++c) {
    scale[c] = (float)(1.0 / stdv[c]);
    shift[c] = (float)(-mean[c] / stdv[c]);
  }
  const int64_t rows_per_task = std::max<int64_t>(1, 4096 / std::max<int64_t>(OW, 1));
  const int64_t tasks_per_img = (OH + rows_per_task - 1) / rows_per_task;
  pybind11::gil_scoped_release nogil;
  pool((int)threads).parallel_for(N * tasks_per_img, [&](int64_t t) {
    const int64_t i = t / tasks_per_img, r0 = (t % tasks_per_img) * rows_per_task;
    const int64_t r1 = std::min(OH, r0 + rows_per_task);
    const int y0 = pr[3 * i], x0 = pr[3 * i + 1], flip = pr[3 * i + 2];
    const uint8_t* im = src[i];
    const int64_t W = Ws[i];
    for (int c = 0; c < 3; ++c) {
      const int sc = to_rgb ? 2 - c : c;               // BGR source channel feeding output channel c
      float* o = dst + ((i * 3 + c) * OH) * OW;
      for (int64_t y = r0; y < r1; ++y) {
        const uint8_t* row = im + ((y0 + y) * W + x0) * 3 + sc;
        float* orow = o + y * OW;
        if (flip) {
          for (int64_t x = 0; x < OW; ++x) orow[x] = row[(OW - 1 - x) * 3] * scale[c] + shift[c];
        } else {
          for (int64_t x = 0; x < OW; ++x) orow[x] = row[x * 3] * scale[c] + shift[c];
        }
      }
    }
  });
}

// Gather fixed-size uint8 records [H, W, 3] at `indices` from a (memory-mapped) record array [R, H, W, 3] into
// a contiguous uint8 batch [N, H, W, 3]; the native side of the indexed record-file dataset.
void gather_records(const torch::Tensor& records, const torch::Tensor& indices, const torch::Tensor& out,
                    int64_t threads) {
  TORCH_CHECK(records.scalar_type() == at::kByte && records.is_contiguous() && !records.is_cuda(),
              "gather_records: records must be contiguous CPU uint8");
  TORCH_CHECK(indices.scalar_type() == at::kLong && indices.dim() == 1, "gather_records: int64 indices");
  TORCH_CHECK(out.scalar_type() == at::kByte && out.is_contiguous() && out.size(0) == indices.size(0),
              "gather_records: out must be uint8 [N, ...]");
  const int64_t R = records.size(0), rec = records.numel() / std::max<int64_t>(R, 1);
  TORCH_CHECK(out.numel() == indices.size(0) * rec, "gather_records: out size mismatch");
  const int64_t* idx = indices.data_ptr<int64_t>();
  for (int64_t i = 0; i < indices.size(0); ++i)
    TORCH_CHECK(idx[i] >= 0 && idx[i] < R, "gather_records: index ", idx[i], " out of range");
  const uint8_t* s = records.data_ptr<uint8_t>();
  uint8_t* d = out.data_ptr<uint8_t>();
  pybind11::gil_scoped_release nogil;
  pool((int)threads).parallel_for(indices.size(0), [&](int64_t i) { std::memcpy(d + i * rec, s + idx[i] * rec, rec); });
}

// ---------------------------------------------------------------------------------------------------------------
// Hadoop SequenceFile of BGR image records (reference S/dataset/DataSet.scala SeqFileFolder + BGRImage.readImage;
// writer dataset/seqfile.py): the whole file is one uint8 tensor, indexed once in C++ so batches are gathered by
// byte offset with the GIL released — no per-record Python on the training data path.
// ---------------------------------------------------------------------------------------------------------------
namespace {
int64_t read_vlong(const uint8_t* b, int64_t n, int64_t& pos) {
  TORCH_CHECK(pos < n, "seqfile: truncated vlong");
  const int8_t first = (int8_t)b[pos++];
  if (first >= -112) return first;
  const bool neg = first < -120;
  const int len = neg ? -(first + 120) : -(first + 112);
  TORCH_CHECK(pos + len <= n, "seqfile: truncated vlong");
  int64_t v = 0;
  for (int i = 0; i < len; ++i) v = (v << 8) | b[pos++];
  return neg ? (v ^ -1) : v;
}
int32_t read_be32(const uint8_t* b, int64_t n, int64_t pos) {
  TORCH_CHECK(pos + 4 <= n, "seqfile: truncated record");
  return (int32_t)(((uint32_t)b[pos] << 24) | ((uint32_t)b[pos + 1] << 16) | ((uint32_t)b[pos + 2] << 8) | b[pos + 3]);
}
}  // namespace

// -> (records int64 [R, 3] = (pixel byte offset, H, W), labels float32 [R]); Text or BytesWritable values holding
// (int32 width, int32 height, BGR bytes), keys "label" or "name\nlabel".
std::vector<torch::Tensor> seqfile_index(const torch::Tensor& buf) {
  TORCH_CHECK(buf.scalar_type() == at::kByte && buf.dim() == 1 && buf.is_contiguous() && !buf.is_cuda(),
              "seqfile_index: buf must be a contiguous CPU uint8 vector");
  const uint8_t* b = buf.data_ptr<uint8_t>();
  const int64_t n = buf.numel();
  TORCH_CHECK(n >= 4 && b[0] == 'S' && b[1] == 'E' && b[2] == 'Q' && b[3] >= 6, "seqfile_index: not a SequenceFile v6");
  int64_t pos = 4;
  std::string cls[2];
  for (int i = 0; i < 2; ++i) {
    const int64_t l = read_vlong(b, n, pos);
    TORCH_CHECK(l >= 0 && pos + l <= n, "seqfile_index: bad class name");
    cls[i].assign((const char*)b + pos, (size_t)l);
    pos += l;
  }
  TORCH_CHECK(pos + 2 <= n && b[pos] == 0 && b[pos + 1] == 0, "seqfile_index: compressed SequenceFiles are not supported");
  pos += 2;
  const int32_t nmeta = read_be32(b, n, pos);
  pos += 4;
  for (int i = 0; i < 2 * nmeta; ++i) {
    const int64_t l = read_vlong(b, n, pos);
    pos += l;
  }
  TORCH_CHECK(pos + 16 <= n, "seqfile_index: truncated header");
  const uint8_t* sync = b + pos;
  pos += 16;
  const bool val_bytes = cls[1] == "org.apache.hadoop.io.BytesWritable";
  const bool key_bytes = cls[0] == "org.apache.hadoop.io.BytesWritable";
  std::vector<int64_t> recs;
  std::vector<float> labels;
  while (pos < n) {
    const int32_t rec_len = read_be32(b, n, pos);
    pos += 4;
    if (rec_len == -1) {
      TORCH_CHECK(pos + 16 <= n && std::memcmp(b + pos, sync, 16) == 0, "seqfile_index: corrupt sync marker at ", pos);
      pos += 16;
      continue;
    }
    const int32_t key_len = read_be32(b, n, pos);
    pos += 4;
    TORCH_CHECK(rec_len >= key_len && key_len >= 0 && pos + rec_len <= n, "seqfile_index: bad record at ", pos);
    // key text -> label (last line)
    int64_t kp = pos, kl;
    if (key_bytes) { kl = read_be32(b, n, kp); kp += 4; } else { kl = read_vlong(b, n, kp); }
    int64_t ls = kp;
    for (int64_t i = kp; i < kp + kl; ++i)
      if (b[i] == '\n') ls = i + 1;
    std::string lab((const char*)b + ls, (size_t)(kp + kl - ls));
    labels.push_back((float)std::strtod(lab.c_str(), nullptr));
    // value -> (w, h, BGR)
    int64_t vp = pos + key_len, vl;
    if (val_bytes) { vl = read_be32(b, n, vp); vp += 4; } else { vl = read_vlong(b, n, vp); }
    TORCH_CHECK(vl >= 8 && vp + vl <= pos + rec_len, "seqfile_index: bad value at ", vp);
    const int32_t w = read_be32(b, n, vp), h = read_be32(b, n, vp + 4);
    TORCH_CHECK(w > 0 && h > 0 && (int64_t)w * h * 3 + 8 <= vl, "seqfile_index: image record larger than its value");
    recs.push_back(vp + 8);
    recs.push_back(h);
    recs.push_back(w);
    pos += rec_len;
  }
  const int64_t R = (int64_t)labels.size();
  auto r = torch::empty({R, 3}, torch::kLong);
  auto l = torch::empty({R}, torch::kFloat);
  if (R) {
    std::memcpy(r.data_ptr<int64_t>(), recs.data(), recs.size() * sizeof(int64_t));
    std::memcpy(l.data_ptr<float>(), labels.data(), labels.size() * sizeof(float));
  }
  return {r, l};
}

// Gather variable-size records: out[dst_off[i] : dst_off[i] + nbytes[i]] = buf[src_off[i] : ...] (parallel memcpy,
// GIL released); out is typically a pinned staging buffer that the device feed copies to the GPU.
void gather_bytes(const torch::Tensor& buf, const torch::Tensor& src_off, const torch::Tensor& nbytes,
                  const torch::Tensor& dst_off, const torch::Tensor& out, int64_t threads) {
  TORCH_CHECK(buf.scalar_type() == at::kByte && buf.is_contiguous() && !buf.is_cuda(), "gather_bytes: uint8 CPU buf");
  TORCH_CHECK(out.scalar_type() == at::kByte && out.is_contiguous() && !out.is_cuda(), "gather_bytes: uint8 CPU out");
  TORCH_CHECK(src_off.scalar_type() == at::kLong && nbytes.scalar_type() == at::kLong && dst_off.scalar_type() == at::kLong &&
                  src_off.is_contiguous() && nbytes.is_contiguous() && dst_off.is_contiguous() &&
                  src_off.numel() == nbytes.numel() && dst_off.numel() == nbytes.numel(),
              "gather_bytes: int64 offset / size vectors of one length");
  const int64_t N = nbytes.numel(), nb = buf.numel(), no = out.numel();
  const int64_t *so = src_off.data_ptr<int64_t>(), *sz = nbytes.data_ptr<int64_t>(), *dof = dst_off.data_ptr<int64_t>();
  for (int64_t i = 0; i < N; ++i)
    TORCH_CHECK(so[i] >= 0 && sz[i] >= 0 && so[i] + sz[i] <= nb && dof[i] >= 0 && dof[i] + sz[i] <= no,
                "gather_bytes: record ", i, " out of range");
  const uint8_t* s = buf.data_ptr<uint8_t>();
  uint8_t* d = out.data_ptr<uint8_t>();
  // 256 KB chunks: a few large images spread over every thread
  constexpr int64_t CH = 256 << 10;
  std::vector<int64_t> first(N + 1, 0);
  for (int64_t i = 0; i < N; ++i) first[i + 1] = first[i] + std::max<int64_t>(1, (sz[i] + CH - 1) / CH);
  pybind11::gil_scoped_release nogil;
  pool((int)threads).parallel_for(first[N], [&](int64_t t) {
    const int64_t i = std::upper_bound(first.begin(), first.end(), t) - first.begin() - 1;
    const int64_t c0 = (t - first[i]) * CH, c1 = std::min(sz[i], c0 + CH);
    if (c1 > c0) std::memcpy(d + dof[i] + c0, s + so[i] + c0, (size_t)(c1 - c0));
  });
}

int64_t pool_size(int64_t threads) { return pool((int)threads).size() + 1; }

}  // namespace bigdl_host

void register_host_runtime(pybind11::module& m) {
  m.def("assemble_batch", &bigdl_host::assemble_batch, "crop/flip/BGR->RGB/normalise uint8 HWC images into an fp32 NCHW batch",
        pybind11::arg("images"), pybind11::arg("params"), pybind11::arg("out"), pybind11::arg("mean"),
        pybind11::arg("std"), pybind11::arg("to_rgb") = true, pybind11::arg("threads") = 0);
  m.def("gather_records", &bigdl_host::gather_records, pybind11::arg("records"), pybind11::arg("indices"),
        pybind11::arg("out"), pybind11::arg("threads") = 0);
  m.def("host_pool_size", &bigdl_host::pool_size, pybind11::arg("threads") = 0);
  m.def("seqfile_index", &bigdl_host::seqfile_index, pybind11::arg("buf"),
        "index a SequenceFile of BGR image records: ((pixel offset, H, W) int64 [R, 3], labels float32 [R])");
  m.def("gather_bytes", &bigdl_host::gather_bytes, pybind11::arg("buf"), pybind11::arg("src_off"),
        pybind11::arg("nbytes"), pybind11::arg("dst_off"), pybind11::arg("out"), pybind11::arg("threads") = 0);
}
