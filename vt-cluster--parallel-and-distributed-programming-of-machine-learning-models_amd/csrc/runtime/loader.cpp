// Native micro-batch producer (the data-loader half of the runtime).
//
// Reference: HF `datasets` (Arrow, C++) feeding `DataCollatorForLanguageModeling` inside the
// HF Trainer's DataLoader workers ([lib]).  Here one C++ worker thread per
// loader gathers the rows of this rank's epoch order from the in-memory token matrix
// ([N, S] int32 + lengths), builds attention masks and causal-LM labels (input_ids with
// padding and pad-id tokens -> -100, the collator's rule incl. B17), and writes them into
// PINNED host tensors, a bounded queue of `prefetch` micro-batches ahead of the consumer.
// The training loop then only issues async H2D copies: no Python-side gather / mask / label
// work or pageable copies on the step's critical path.
//
//   L = mift._C.TokenLoader(ids, lengths, pad_id, micro_batch, prefetch, pin)
//   L.start(order, first_micro_batch)   # order: int64 row indices (DP shard, shuffled or not)
//   L.next() -> [input_ids, attention_mask, labels] (int64 [b, S]) or [] at the end
#include <torch/extension.h>

#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace {

class TokenLoader {
 public:
  TokenLoader(at::Tensor ids, at::Tensor lengths, int64_t pad_id, int64_t micro_batch, int64_t prefetch, bool pin)
      : ids_(ids.contiguous()), len_(lengths.contiguous()), pad_(pad_id), mb_(micro_batch),
        cap_(std::max<int64_t>(1, prefetch)), pin_(pin) {
    TORCH_CHECK(!ids_.is_cuda() && ids_.dim() == 2 && ids_.scalar_type() == at::kInt, "TokenLoader: ids int32 [N,S] CPU");
    TORCH_CHECK(!len_.is_cuda() && len_.scalar_type() == at::kInt && len_.numel() == ids_.size(0),
                "TokenLoader: lengths int32 [N] CPU");
    TORCH_CHECK(mb_ >= 1, "TokenLoader: micro_batch >= 1");
  }
  ~TokenLoader() { stop(); }

  void start(at::Tensor order, int64_t first_mb) {
    stop();
    TORCH_CHECK(!order.is_cuda() && order.scalar_type() == at::kLong && order.dim() == 1, "TokenLoader: order int64 [n]");
    order_ = order.contiguous();
    const int64_t n = order_.numel();
    const int64_t nmb = (n + mb_ - 1) / mb_;
    const int64_t N = ids_.size(0);
    const int64_t* o = order_.data_ptr<int64_t>();
    for (int64_t i = 0; i < n; ++i) TORCH_CHECK(o[i] >= 0 && o[i] < N, "TokenLoader: row index out of range");
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.clear();
      done_ = false;
      quit_ = false;
    }
    worker_ = std::thread([this, first_mb, nmb, n] { run(first_mb, nmb, n); });
  }

  std::vector<at::Tensor> next() {
    std::unique_lock<std::mutex> lk(mu_);
    {
      pybind11::gil_scoped_release nogil;
      cv_.wait(lk, [this] { return !q_.empty() || done_; });
    }
    if (q_.empty()) {
      if (!err_.empty()) {
        std::string e = err_;
        err_.clear();
        TORCH_CHECK(false, "TokenLoader worker failed: ", e);
      }
      return {};
    }
    auto item = std::move(q_.front());
    q_.pop_front();
    cv_.notify_all();
    return item;
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) {
      if (PyGILState_Check()) {
        pybind11::gil_scoped_release nogil;
        worker_.join();
      } else {
        worker_.join();
      }
    }
  }

 private:
  void run(int64_t first_mb, int64_t nmb, int64_t n) {
    try {
      const int64_t S = ids_.size(1);
      const int32_t* ids = ids_.data_ptr<int32_t>();
      const int32_t* lens = len_.data_ptr<int32_t>();
      const int64_t* order = order_.data_ptr<int64_t>();
      auto opt = at::TensorOptions().dtype(at::kLong).pinned_memory(pin_);
      for (int64_t j = first_mb; j < nmb; ++j) {
        const int64_t r0 = j * mb_, b = std::min(mb_, n - r0);
        at::Tensor in = at::empty({b, S}, opt), am = at::empty({b, S}, opt), lab = at::empty({b, S}, opt);
        int64_t* pi = in.data_ptr<int64_t>();
        int64_t* pm = am.data_ptr<int64_t>();
        int64_t* pl = lab.data_ptr<int64_t>();
        for (int64_t i = 0; i < b; ++i) {
          const int64_t row = order[r0 + i];
          const int32_t* src = ids + row * S;
          const int64_t L = lens[row];
          for (int64_t s = 0; s < S; ++s) {
            const int64_t t = src[s];
            const int64_t valid = s < L ? 1 : 0;
            pi[i * S + s] = t;
            pm[i * S + s] = valid;
            pl[i * S + s] = (valid && t != pad_) ? t : -100;
          }
        }
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return (int64_t)q_.size() < cap_ || quit_; });
        if (quit_) return;
        q_.push_back({in, am, lab});
        cv_.notify_all();
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(mu_);
      err_ = e.what();
    }
    std::lock_guard<std::mutex> g(mu_);
    done_ = true;
    cv_.notify_all();
  }

  at::Tensor ids_, len_, order_;
  int64_t pad_, mb_, cap_;
  bool pin_;
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::vector<at::Tensor>> q_;
  bool done_ = false, quit_ = false;
  std::string err_;
};

}  // namespace

void mift_bind_runtime(pybind11::module& m) {
  pybind11::class_<TokenLoader>(m, "TokenLoader",
                                "native prefetching micro-batch producer (pinned input_ids / attention_mask / labels)")
      .def(pybind11::init<at::Tensor, at::Tensor, int64_t, int64_t, int64_t, bool>(), pybind11::arg("ids"),
           pybind11::arg("lengths"), pybind11::arg("pad_id"), pybind11::arg("micro_batch"),
           pybind11::arg("prefetch") = 4, pybind11::arg("pin") = true)
      .def("start", &TokenLoader::start, pybind11::arg("order"), pybind11::arg("first_micro_batch") = 0)
      .def("next", &TokenLoader::next)
      .def("stop", &TokenLoader::stop);
}
