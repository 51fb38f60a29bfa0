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

int64_t pool_size(int64_t threads) { return pool((int)threads).size() + 1; }

}  // namespace bigdl_host

void register_host_runtime(pybind11::module& m) {
  m.def("assemble_batch", &bigdl_host::assemble_batch, "crop/flip/BGR->RGB/normalise uint8 HWC images into an fp32 NCHW batch",
        pybind11::arg("images"), pybind11::arg("params"), pybind11::arg("out"), pybind11::arg("mean"),
        pybind11::arg("std"), pybind11::arg("to_rgb") = true, pybind11::arg("threads") = 0);
  m.def("gather_records", &bigdl_host::gather_records, pybind11::arg("records"), pybind11::arg("indices"),
        pybind11::arg("out"), pybind11::arg("threads") = 0);
  m.def("host_pool_size", &bigdl_host::pool_size, pybind11::arg("threads") = 0);
}
