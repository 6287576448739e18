// pybind11 bindings of the host runtime (module `_runtime`).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_manager.h"
#include "scheduler.h"

namespace py = pybind11;
using namespace akap_rt;

template <typename T>
static T* ptr_of(py::dict& d, const char* k, size_t min_elems) {
  auto a = d[k].cast<py::array_t<T, py::array::c_style>>();
  if ((size_t)a.size() < min_elems) throw std::invalid_argument(std::string("buffer too small: ") + k);
  return a.mutable_data();
}

static BatchBuffers batch_buffers(const Scheduler& s, py::dict bufs) {
  const auto& c = s.config();
  BatchBuffers b{};
  b.cap_tokens = bufs["input_ids"].cast<py::array>().size();
  b.input_ids = ptr_of<int64_t>(bufs, "input_ids", b.cap_tokens);
  b.positions = ptr_of<int64_t>(bufs, "positions", b.cap_tokens);
  b.slots = ptr_of<int64_t>(bufs, "slots", b.cap_tokens);
  b.seq_lens = ptr_of<int32_t>(bufs, "seq_lens", c.max_num_seqs);
  b.q_start = ptr_of<int32_t>(bufs, "q_start", c.max_num_seqs + 1);
  b.block_tables =
      ptr_of<int32_t>(bufs, "block_tables", (size_t)c.max_num_seqs * c.max_blocks_per_seq);
  b.cap_tiles = bufs["tile_seq"].cast<py::array>().size();
  b.tile_seq = ptr_of<int32_t>(bufs, "tile_seq", b.cap_tiles);
  b.tile_row = ptr_of<int32_t>(bufs, "tile_row", b.cap_tiles);
  b.logits_idx = ptr_of<int64_t>(bufs, "logits_idx", c.max_num_seqs);
  b.req_ids = ptr_of<int64_t>(bufs, "req_ids", c.max_num_seqs);
  b.sample_mask = ptr_of<int32_t>(bufs, "sample_mask", c.max_num_seqs);
  b.temperature = ptr_of<float>(bufs, "temperature", c.max_num_seqs);
  b.top_p = ptr_of<float>(bufs, "top_p", c.max_num_seqs);
  b.top_k = ptr_of<int32_t>(bufs, "top_k", c.max_num_seqs);
  b.seeds = ptr_of<int64_t>(bufs, "seeds", c.max_num_seqs);
  b.steps = ptr_of<int32_t>(bufs, "steps", c.max_num_seqs);
  b.tail_slot = bufs.contains("tail_slot") ? ptr_of<int32_t>(bufs, "tail_slot", b.cap_tokens)
                                           : nullptr;
  return b;
}

static py::dict step_info(const StepInfo& i) {
  py::dict d;
  d["is_prefill"] = i.is_prefill;
  d["num_seqs"] = i.num_seqs;
  d["num_tokens"] = i.num_tokens;
  d["num_tiles"] = i.num_tiles;
  d["num_samples"] = i.num_samples;
  d["max_seq_len"] = i.max_seq_len;
  d["num_preempted"] = i.num_preempted;
  d["num_decode"] = i.num_decode;
  d["tile_rows"] = i.tile_rows;
  return d;
}

#ifndef AKAP_RT_HASH
#define AKAP_RT_HASH "unknown"
#endif

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "MI355X serving engine host runtime: paged KV block manager + batch scheduler";
  // digest of the runtime sources this module was compiled from (build_ext.runtime_tree_hash)
  m.def("build_hash", [] { return std::string(AKAP_RT_HASH); });

  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("enable_prefix_cache") = true)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("num_free", &BlockManager::num_free)
      .def("usage", &BlockManager::usage)
      .def("allocate", &BlockManager::allocate)
      .def("free_blocks", &BlockManager::free_blocks)
      .def("register_full", &BlockManager::register_full)
      .def("output_tokens", [](const Scheduler& s, int64_t id) {
        auto r = s.get(id);
        std::vector<int32_t> out;
        if (r) out.assign(r->tokens.begin() + r->num_prompt, r->tokens.end());
        return out;
      })
      .def("reset_prefix_cache", &BlockManager::reset_prefix_cache)
      .def("match_prefix",
           [](BlockManager& bm, const std::vector<int32_t>& toks, int max_tokens) {
             std::vector<int32_t> b;
             std::vector<uint64_t> h;
             int n = bm.match_prefix(toks, max_tokens, b, h);
             return py::make_tuple(n, b, h);
           })
      .def_static("hash_block", [](uint64_t parent, const std::vector<int32_t>& t) {
        return BlockManager::hash_block(parent, t.data(), (int)t.size());
      });

  py::class_<SchedConfig>(m, "SchedConfig")
      .def(py::init<>())
      .def_readwrite("max_num_seqs", &SchedConfig::max_num_seqs)
      .def_readwrite("max_num_batched_tokens", &SchedConfig::max_num_batched_tokens)
      .def_readwrite("max_model_len", &SchedConfig::max_model_len)
      .def_readwrite("block_size", &SchedConfig::block_size)
      .def_readwrite("gqa_group", &SchedConfig::gqa_group)
      .def_readwrite("tile_rows", &SchedConfig::tile_rows)
      .def_readwrite("tile_rows_short", &SchedConfig::tile_rows_short)
      .def_readwrite("short_rows", &SchedConfig::short_rows)
      .def_readwrite("eos_id", &SchedConfig::eos_id)
      .def_readwrite("max_blocks_per_seq", &SchedConfig::max_blocks_per_seq)
      .def_readwrite("mixed_batching", &SchedConfig::mixed_batching)
      .def_readwrite("mix_backlog_steps", &SchedConfig::mix_backlog_steps)
      .def_readwrite("max_decode_stall_steps", &SchedConfig::max_decode_stall_steps)
      .def_readwrite("held_kv_ttl_s", &SchedConfig::held_kv_ttl_s)
      .def_readwrite("num_tail_slots", &SchedConfig::num_tail_slots);

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<const SchedConfig&, int, bool>(), py::arg("config"), py::arg("num_blocks"),
           py::arg("prefix_cache") = true)
      // the prompt as a contiguous int32 array: one memcpy instead of a per-element conversion
      // of a Python list (a 512-token prompt: ~25 us -> ~1 us, which the bulk admission of a
      // 256-request wave pays 256 times before its first step).  Registered first: a list
      // fails this overload's no-convert pass and takes the std::vector one below
      .def(
          "add_request",
          [](Scheduler& s, int64_t id,
             py::array_t<int32_t, py::array::c_style | py::array::forcecast> prompt,
             int max_tokens, int min_tokens, bool ignore_eos, const std::vector<int32_t>& stop_ids,
             float temperature, float top_p, int top_k, int64_t seed, bool stream) {
            const int32_t* d = prompt.data();
            s.add_request(id, std::vector<int32_t>(d, d + prompt.size()), max_tokens, min_tokens,
                          ignore_eos, stop_ids, temperature, top_p, top_k, seed, stream);
          },
          py::arg("id"), py::arg("prompt"), py::arg("max_tokens"), py::arg("min_tokens") = 0,
          py::arg("ignore_eos") = false, py::arg("stop_ids") = std::vector<int32_t>{},
          py::arg("temperature") = 0.f, py::arg("top_p") = 1.f, py::arg("top_k") = 0,
          py::arg("seed") = 0, py::arg("stream") = false)
      .def("add_request", &Scheduler::add_request, py::arg("id"), py::arg("prompt"),
           py::arg("max_tokens"), py::arg("min_tokens") = 0, py::arg("ignore_eos") = false,
           py::arg("stop_ids") = std::vector<int32_t>{}, py::arg("temperature") = 0.f,
           py::arg("top_p") = 1.f, py::arg("top_k") = 0, py::arg("seed") = 0,
           py::arg("stream") = false)
      .def("abort_request", &Scheduler::abort_request)
      .def("release", &Scheduler::release)
      .def("schedule",
           [](Scheduler& s, py::dict bufs) {
             BatchBuffers b = batch_buffers(s, bufs);
             StepInfo i;
             {
               py::gil_scoped_release nogil;
               i = s.schedule(b);
             }
             return step_info(i);
           })
      .def("schedule_lookahead",
           [](Scheduler& s, py::dict bufs) {
             BatchBuffers b = batch_buffers(s, bufs);
             int64_t* src = ptr_of<int64_t>(bufs, "src_rows", s.config().max_num_seqs);
             StepInfo i;
             {
               py::gil_scoped_release nogil;
               i = s.schedule_lookahead(b, src);
             }
             return step_info(i);
           })
      .def("update",
           [](Scheduler& s, py::array_t<int64_t, py::array::c_style> toks) {
             std::vector<int64_t> ids;
             std::vector<int32_t> t, f, first;
             s.update(toks.data(), (int)toks.size(), ids, t, f, first);
             return py::make_tuple(ids, t, f, first);
           })
      .def_property_readonly("num_waiting", &Scheduler::num_waiting)
      .def_property_readonly("num_running", &Scheduler::num_running)
      .def("has_work", &Scheduler::has_work)
      .def("block_table", &Scheduler::block_table)
      .def("kv_usage", [](const Scheduler& s) { return s.blocks().usage(); })
      .def("num_free_blocks", [](const Scheduler& s) { return s.blocks().num_free(); })
      .def("prefix_stats", [](const Scheduler& s) {
        return py::make_tuple(s.blocks().prefix_hits(), s.blocks().prefix_queries());
      })
      .def("output_tokens", [](const Scheduler& s, int64_t id) {
        auto r = s.get(id);
        std::vector<int32_t> out;
        if (r) out.assign(r->tokens.begin() + r->num_prompt, r->tokens.end());
        return out;
      })
      .def("reset_prefix_cache", [](Scheduler& s) { s.blocks_mut().reset_prefix_cache(); })
      .def("set_hold_kv", &Scheduler::set_hold_kv)
      .def("held_blocks", &Scheduler::held_blocks)
      .def("free_held", &Scheduler::free_held)
      .def("take_held", &Scheduler::take_held)
      .def("finish_transfer", &Scheduler::finish_transfer)
      .def_property_readonly("num_in_transfer", &Scheduler::num_in_transfer)
      .def_property_readonly("last_appended", &Scheduler::last_appended)
      .def_property_readonly("num_held", &Scheduler::num_held)
      .def("expire_held", &Scheduler::expire_held, py::arg("now_s"))
      .def_static("now_s", &Scheduler::now_s)
      .def_property_readonly("held_expired_total", &Scheduler::held_expired_total)
      .def("reserve_prefilled", &Scheduler::reserve_prefilled, py::arg("id"), py::arg("tokens"),
           py::arg("num_prompt"), py::arg("max_tokens"), py::arg("min_tokens") = 0,
           py::arg("ignore_eos") = false, py::arg("stop_ids") = std::vector<int32_t>{},
           py::arg("temperature") = 0.f, py::arg("top_p") = 1.f, py::arg("top_k") = 0,
           py::arg("seed") = 0, py::arg("stream") = false)
      .def("activate", &Scheduler::activate)
      .def("set_first_token", &Scheduler::set_first_token)
      .def("tail_slot", &Scheduler::tail_slot)
      .def_property_readonly("num_free_tail_slots", &Scheduler::num_free_tail_slots)
      .def_property_readonly("total_preemptions", &Scheduler::total_preemptions)
      .def("request_info", [](const Scheduler& s, int64_t id) -> py::object {
        auto r = s.get(id);
        if (!r) return py::none();
        py::dict d;
        d["num_prompt"] = r->num_prompt;
        d["num_tokens"] = (int)r->tokens.size();
        d["num_computed"] = r->num_computed;
        d["num_cached"] = r->num_cached;
        d["status"] = r->status;
        d["finish"] = r->finish;
        d["num_preempt"] = r->num_preempt;
        d["tokens"] = r->tokens;
        d["stream"] = r->stream;
        return d;
      });
}
