// ai4e_core — native control plane of the MI355X serving platform (pybind11 bindings).
//
// Replaces the reference's Redis-backed task cache + Service Bus transport + per-endpoint
// dispatcher functions (ProcessManager/CacheManager/CacheConnectorUpsert.cs:40-213,
// CacheConnectorGet.cs:27-73, BackendQueueProcessor/BackendQueueProcessor.cs:27-81,
// RequestReporter/CurrentProcessingUpsert.cs:99-110, Libraries/QueueLogger.cs:21-47):
//
//   TaskStore      task_store.h     records, per-(path,state) indexes, _ORIG bodies, counters,
//                                   attached results, TTL eviction, journal
//   DispatchQueue  dispatch_queue.h peek-lock FIFO with abandon/redelivery/dead-letter + batching
//   SlotRing       slot_ring.h      payload-ring slot allocator (one partition per ingest process)
//   NodeScheduler  scheduler.h      queue -> batch -> GPU worker process -> results, GIL-free
//
// Every blocking call releases the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "dispatch_queue.h"
#include "jpeg_coef.h"
#define AI4E_HD
#include "jpeg_span.h"
#include "scheduler.h"
#include "slot_ring.h"
#include "task_store.h"

namespace py = pybind11;
using namespace ai4e;

namespace {

py::dict view_dict(const TaskStore::View& v) {
  py::dict d;
  d["TaskId"] = v.id;
  d["Timestamp"] = v.timestamp;
  d["Status"] = v.status;
  d["BackendStatus"] = v.backend_status;
  d["Endpoint"] = v.endpoint;
  d["Body"] = py::none();
  d["PublishToGrid"] = v.pub;
  d["EndpointPath"] = v.path;
  return d;
}

// Build a ResultBatch from Python buffers (the in-process GPU worker path).
std::shared_ptr<const ResultBatch> make_batch(const py::bytes& rows, uint32_t row_bytes, const std::vector<double>& stage,
                                              int worker) {
  auto r = std::make_shared<ResultBatch>();
  r->data = rows;
  r->row_bytes = row_bytes;
  for (size_t i = 0; i < stage.size() && i < 5; ++i) r->stage[i] = stage[i];
  r->worker = worker;
  return r;
}

}  // namespace

PYBIND11_MODULE(_ai4e_core, m) {
  m.doc() = "Native task store, dispatch queue, slot ring and node scheduler of the MI355X AI4E platform";
  m.def("dotnet_timestamp", &dotnet_timestamp);
  m.def("absolute_path", &absolute_path);
  m.def("uuid4", []() {
    static Uuid4 u;
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    return u.next();
  });
  m.def("mono_now", &mono_now);

  py::class_<TaskStore, std::shared_ptr<TaskStore>>(m, "TaskStore")
      .def(py::init<std::string, size_t>(), py::arg("journal_path") = "", py::arg("nshards") = 8)
      .def_property_readonly("nshards", &TaskStore::nshards)
      .def("upsert", &TaskStore::upsert, py::arg("task_id"), py::arg("status"), py::arg("backend_status"),
           py::arg("endpoint"), py::arg("body") = std::nullopt, py::arg("publish_to_grid") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("create_many", &TaskStore::create_many, py::arg("endpoint"), py::arg("n"), py::arg("status") = "created",
           py::arg("trace") = "", py::call_guard<py::gil_scoped_release>())
      .def("create_many_in", &TaskStore::create_many_in, py::arg("shard"), py::arg("endpoint"), py::arg("n"),
           py::arg("status") = "created", py::arg("trace") = "", py::call_guard<py::gil_scoped_release>())
      .def("shard_index", &TaskStore::shard_index)
      .def("create_ids", &TaskStore::create_ids, py::arg("endpoint"), py::arg("ids"), py::arg("status") = "created",
           py::arg("trace") = "", py::call_guard<py::gil_scoped_release>())
      .def("transition_many", &TaskStore::transition_many, py::arg("ids"), py::arg("backend_status"),
           py::arg("status"), py::call_guard<py::gil_scoped_release>())
      .def("retarget_many", &TaskStore::retarget_many, py::arg("ids"), py::arg("endpoint"), py::arg("status"),
           py::call_guard<py::gil_scoped_release>())
      .def(
          "finish_batch",
          [](TaskStore& s, const std::vector<std::string>& ids, const py::bytes& rows, uint32_t row_bytes,
             const std::vector<uint8_t>& ok, const std::vector<double>& stage, int worker, const std::string& status_ok,
             const std::string& status_fail) {
            auto b = make_batch(rows, row_bytes, stage, worker);
            py::gil_scoped_release rel;
            s.finish_many(ids, b, ok, status_ok, status_fail);
          },
          py::arg("ids"), py::arg("rows"), py::arg("row_bytes"), py::arg("ok") = std::vector<uint8_t>{},
          py::arg("stage") = std::vector<double>{}, py::arg("worker") = -1, py::arg("status_ok") = "completed",
          py::arg("status_fail") = "Task failed - try again")
      .def("set_status_text", &TaskStore::set_status_text, py::call_guard<py::gil_scoped_release>())
      .def("set_trace", &TaskStore::set_trace, py::call_guard<py::gil_scoped_release>())
      .def("get", &TaskStore::get, py::call_guard<py::gil_scoped_release>())
      .def("get_record",
           [](TaskStore& s, const std::string& id) -> py::object {
             std::optional<TaskStore::View> v;
             {
               py::gil_scoped_release rel;
               v = s.view(id);
             }
             if (!v) return py::none();
             return view_dict(*v);
           })
      // Model output row of a finished task (bytes) or None.
      .def("result",
           [](TaskStore& s, const std::string& id) -> py::object {
             std::optional<TaskStore::View> v;
             {
               py::gil_scoped_release rel;
               v = s.view(id);
             }
             if (!v || !v->res || v->backend_status != "completed") return py::none();
             const auto& b = *v->res;
             const size_t off = static_cast<size_t>(v->row) * b.row_bytes;
             if (off + b.row_bytes > b.data.size()) return py::none();
             return py::bytes(b.data.data() + off, b.row_bytes);
           })
      // Per-task stage trace: accept/created, dispatched/running, worker recv/launch/gpu-done,
      // GPU h2d/compute ms, finished (CLOCK_MONOTONIC seconds) + the B3 trace context.
      .def("trace",
           [](TaskStore& s, const std::string& id) -> py::object {
             std::optional<TaskStore::View> v;
             {
               py::gil_scoped_release rel;
               v = s.view(id);
             }
             if (!v) return py::none();
             py::dict d;
             d["TaskId"] = v->id;
             d["BackendStatus"] = v->backend_status;
             d["trace"] = v->trace;
             d["t_created"] = v->t_created;
             d["t_running"] = v->t_running;
             d["t_finished"] = v->t_finished;
             if (v->res) {
               d["worker"] = v->res->worker;
               d["t_worker_recv"] = v->res->stage[0];
               d["t_worker_launch"] = v->res->stage[1];
               d["t_worker_done"] = v->res->stage[2];
               d["gpu_h2d_ms"] = v->res->stage[3];
               d["gpu_compute_ms"] = v->res->stage[4];
             }
             return d;
           })
      .def("get_orig_body", &TaskStore::get_orig_body)
      .def("latencies", &TaskStore::latencies, py::arg("ids"), py::arg("to_running") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("latencies_window", &TaskStore::latencies_window, py::arg("path"), py::arg("t0"), py::arg("t1"),
           py::call_guard<py::gil_scoped_release>())
      .def("zcard", &TaskStore::zcard)
      .def("zrange", &TaskStore::zrange, py::arg("key"), py::arg("limit") = static_cast<size_t>(-1))
      .def("keys_with_suffix", &TaskStore::keys_with_suffix)
      .def("incrby", &TaskStore::incrby)
      .def("get_counter", &TaskStore::get_counter)
      .def("counters", &TaskStore::counters)
      .def("evict_finished", &TaskStore::evict_finished, py::arg("max_age_s"),
           py::arg("max_finished") = static_cast<size_t>(SIZE_MAX), py::call_guard<py::gil_scoped_release>())
      .def("size", &TaskStore::size)
      .def("flush", &TaskStore::flush)
      .def("journaled", &TaskStore::journaled)
      .def("replay", [](TaskStore& s, const std::string& path) {
        py::module_ json = py::module_::import("json");
        return s.replay(path, [&](const std::string& line, TaskStore::JournalLine& jl) {
          try {
            py::dict d = json.attr("loads")(line);
            jl.id = d["TaskId"].cast<std::string>();
            jl.timestamp = d["Timestamp"].cast<std::string>();
            jl.status = d["Status"].cast<std::string>();
            jl.backend_status = d["BackendStatus"].cast<std::string>();
            jl.endpoint = d["Endpoint"].cast<std::string>();
            jl.pub = d["PublishToGrid"].cast<bool>();
            jl.score = d.contains("_score") ? d["_score"].cast<double>() : 0.0;
            if (d.contains("_orig") && !d["_orig"].is_none()) jl.orig = d["_orig"].cast<std::string>();
            return true;
          } catch (...) {
            return false;  // torn tail line after a crash
          }
        });
      });

  py::class_<Message>(m, "Message")
      .def_readonly("seq", &Message::seq)
      .def_readonly("task_id", &Message::task_id)
      .def_readonly("ref", &Message::ref)
      .def_property_readonly("body", [](const Message& msg) { return py::bytes(msg.body); })
      .def_readonly("delivery_count", &Message::delivery_count)
      .def_readonly("enqueued_at", &Message::enqueued_at);

  py::class_<DispatchQueue, std::shared_ptr<DispatchQueue>>(m, "DispatchQueue")
      .def(py::init<std::string, int, double, size_t>(), py::arg("name"), py::arg("max_delivery_count") = 1440,
           py::arg("lock_duration_s") = 300.0, py::arg("max_size") = 0)
      .def_property_readonly("name", &DispatchQueue::name)
      .def("send", &DispatchQueue::send, py::arg("task_id"), py::arg("ref") = -1, py::arg("body") = "",
           py::call_guard<py::gil_scoped_release>())
      .def("send_many", &DispatchQueue::send_many, py::arg("ids"), py::arg("refs") = std::vector<int64_t>{},
           py::call_guard<py::gil_scoped_release>())
      .def("receive", &DispatchQueue::receive, py::arg("max_n") = 1, py::arg("timeout_s") = 0.0,
           py::arg("linger_s") = 0.0, py::call_guard<py::gil_scoped_release>())
      // Batch receive without per-message objects: (task_ids, refs, seqs).
      .def(
          "receive_batch",
          [](DispatchQueue& q, size_t max_n, double timeout_s, double linger_s) {
            std::vector<Message> ms;
            {
              py::gil_scoped_release rel;
              ms = q.receive(max_n, timeout_s, linger_s);
            }
            std::vector<std::string> ids;
            std::vector<int64_t> refs;
            std::vector<uint64_t> seqs;
            ids.reserve(ms.size());
            refs.reserve(ms.size());
            seqs.reserve(ms.size());
            for (auto& x : ms) {
              ids.push_back(std::move(x.task_id));
              refs.push_back(x.ref);
              seqs.push_back(x.seq);
            }
            return py::make_tuple(ids, refs, seqs);
          },
          py::arg("max_n") = 1, py::arg("timeout_s") = 0.0, py::arg("linger_s") = 0.0)
      .def("complete", &DispatchQueue::complete, py::call_guard<py::gil_scoped_release>())
      .def("abandon", &DispatchQueue::abandon, py::arg("seq"), py::arg("delay_s") = 0.0,
           py::call_guard<py::gil_scoped_release>())
      .def("take_deadletters", &DispatchQueue::take_deadletters)
      .def("close", &DispatchQueue::close)
      .def("stats",
           [](DispatchQueue& q) {
             auto s = q.stats();
             py::dict d;
             d["name"] = q.name();
             d["ready"] = s.ready;
             d["scheduled"] = s.scheduled;
             d["inflight"] = s.inflight;
             d["deadlettered"] = s.deadlettered;
             d["sent"] = s.sent;
             return d;
           })
      .def("depth", &DispatchQueue::depth)
      .def("set_lock_duration", &DispatchQueue::set_lock_duration, py::arg("seconds"))
      .def_property_readonly("lock_duration", &DispatchQueue::lock_duration);

  py::class_<SlotRing, std::shared_ptr<SlotRing>>(m, "SlotRing")
      .def(py::init<int64_t, int64_t>(), py::arg("nslots"), py::arg("base") = 0)
      .def("alloc", &SlotRing::alloc, py::arg("n"), py::arg("timeout_s") = -1.0,
           py::call_guard<py::gil_scoped_release>())
      .def("free", &SlotRing::free, py::call_guard<py::gil_scoped_release>())
      .def("owns", &SlotRing::owns)
      .def("used", &SlotRing::used)
      .def("close", &SlotRing::close)
      .def_property_readonly("capacity", &SlotRing::capacity)
      .def_property_readonly("base", &SlotRing::base);

  // Huffman-decode a baseline JPEG into the compact coefficient layout of csrc/core/jpeg_coef.h at address `out`
  // (capacity `cap` bytes; e.g. a payload-ring slot). Returns (status, bytes used); status 0 ok, 1 unsupported
  // (progressive / 12-bit / non-interleaved: decode on the CPU instead), 2 corrupt, 3 does not fit.
  m.def(
      "jpeg_coef_decode",
      [](py::bytes data, uintptr_t out, size_t cap) {
        std::string_view v(data);
        size_t used = 0;
        int st;
        {
          py::gil_scoped_release rel;
          JpegCoefDecoder dec;
          st = dec.decode(reinterpret_cast<const uint8_t*>(v.data()), v.size(), reinterpret_cast<uint8_t*>(out), cap,
                          &used);
        }
        return py::make_tuple(st, used);
      },
      py::arg("data"), py::arg("out"), py::arg("cap"));
  m.attr("JPEG_COEF_HEADER_BYTES") = sizeof(JpegCoefHeader);
  // Headers, GPU Huffman tables and the unstuffed scan (JpegScanHeader layout) for the on-GPU decoder
  // (csrc/kernels/jpeg.hip); same status codes (restart intervals: 1, decode on the CPU).
  m.def(
      "jpeg_scan_prepare",
      [](py::bytes data, uintptr_t out, size_t cap) {
        std::string_view v(data);
        size_t used = 0;
        int st;
        {
          py::gil_scoped_release rel;
          JpegCoefDecoder dec;
          st = dec.prepare(reinterpret_cast<const uint8_t*>(v.data()), v.size(), reinterpret_cast<uint8_t*>(out), cap,
                           &used);
        }
        return py::make_tuple(st, used);
      },
      py::arg("data"), py::arg("out"), py::arg("cap"));
  m.attr("JPEG_SCAN_HEADER_BYTES") = sizeof(JpegScanHeader);
  // Sequential CPU decode of a prepared frame (address `src`, `size` bytes) into int16 [nblocks][64] at `out` (MCU
  // order, natural order, DC undifferenced, not dequantised): the GPU kernels' own span decoder run as one span. For
  // workers on CPU devices and tests. Returns 0 ok, 2 corrupt.
  m.def(
      "jpeg_scan_coefs",
      [](uintptr_t src, size_t size, uintptr_t out) {
        py::gil_scoped_release rel;
        const auto* H = reinterpret_cast<const JpegScanHeader*>(src);
        if (size < sizeof(JpegScanHeader) || H->magic != kJpegScanMagic || H->bpm == 0 || H->bpm > 16 ||
            sizeof(JpegScanHeader) + H->scan_bytes + kJpegScanPad > size)
          return 2;
        static const uint8_t zz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                       12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                       35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                       58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
        std::vector<uint32_t> lut(4u << kGpuLook);
        for (int t = 0; t < 2; ++t) {
          std::memcpy(&lut[static_cast<size_t>(t) << kGpuLook], H->dc[t].fast, sizeof(H->dc[t].fast));
          std::memcpy(&lut[static_cast<size_t>(2 + t) << kGpuLook], H->ac[t].fast, sizeof(H->ac[t].fast));
        }
        uint8_t nat[80], btab[16] = {};
        for (int i = 0; i < 80; ++i) nat[i] = i < 64 ? zz[i] : 63;
        for (uint32_t k = 0; k < H->bpm; ++k) {
          const int c = H->blk_comp[k] < 3 ? H->blk_comp[k] : 0;
          btab[k] = static_cast<uint8_t>((H->comp[c][6] & 1) | ((H->comp[c][7] & 1) << 2) | (c << 4));
        }
        const auto* words = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(src) +
                                                              sizeof(JpegScanHeader));
        JSpanTables T{lut.data(), H->dc, btab, nat, words,
                      static_cast<uint32_t>((H->scan_bytes + kJpegScanPad) / 4), static_cast<int>(H->bpm)};
        auto* coef = reinterpret_cast<int16_t*>(out);
        std::memset(coef, 0, static_cast<size_t>(H->nblocks) * 128);
        const int32_t pred[3] = {0, 0, 0};
        JSpanResult r;
        std::vector<uint8_t> blen(H->nblocks);
        jspan_decode<true>(T, 0, 0, 0, H->total_bits, r, coef, 0, pred, static_cast<int32_t>(H->nblocks), blen.data());
        int16_t blk[64];  // zigzag -> natural order, in place per block
        for (uint32_t q = 0; q < H->nblocks; ++q) {
          int16_t* b = coef + static_cast<size_t>(q) * 64;
          for (int k = 0; k < 64; ++k) blk[zz[k]] = b[k];
          std::memcpy(b, blk, sizeof(blk));
        }
        return (r.bad || r.nblk < static_cast<int32_t>(H->nblocks)) ? 2 : 0;
      },
      py::arg("src"), py::arg("size"), py::arg("out"));

  py::class_<NodeScheduler, std::shared_ptr<NodeScheduler>>(m, "NodeScheduler")
      .def(py::init([](std::shared_ptr<TaskStore> store, std::shared_ptr<DispatchQueue> queue, std::string endpoint,
                       int64_t ring_slots, size_t max_batch, double linger_s, int depth, double retry_delay_s,
                       double hb_timeout_s, double poll_s, double busy_linger_s) {
             SchedConfig c;
             c.max_batch = max_batch;
             c.linger_s = linger_s;
             c.busy_linger_s = busy_linger_s;
             c.depth = depth;
             c.retry_delay_s = retry_delay_s;
             c.hb_timeout_s = hb_timeout_s;
             c.poll_s = poll_s;
             return std::make_shared<NodeScheduler>(std::move(store), std::move(queue), std::move(endpoint),
                                                    ring_slots, c);
           }),
           py::arg("store"), py::arg("queue"), py::arg("endpoint"), py::arg("ring_slots"), py::arg("max_batch") = 250,
           py::arg("linger_s") = 0.0005, py::arg("depth") = 2, py::arg("retry_delay_s") = 1.0,
           py::arg("hb_timeout_s") = 10.0, py::arg("poll_s") = 0.02, py::arg("busy_linger_s") = 0.0)
      .def("add_local_ring", &NodeScheduler::add_local_ring)
      .def("add_remote_partition", &NodeScheduler::add_remote_partition)
      .def("set_stage_endpoints", &NodeScheduler::set_stage_endpoints)
      .def("set_store_shards", &NodeScheduler::set_store_shards)
      .def("enable_completion_feed", &NodeScheduler::enable_completion_feed)
      .def("attach", &NodeScheduler::attach, py::arg("rank"), py::arg("fd"), py::arg("dispatch") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("detach", &NodeScheduler::detach, py::arg("rank"), py::arg("timeout_s") = 30.0,
           py::call_guard<py::gil_scoped_release>())
      .def("wait_failed", &NodeScheduler::wait_failed, py::arg("timeout_s") = 0.0,
           py::call_guard<py::gil_scoped_release>())
      .def("submit", &NodeScheduler::submit, py::arg("slots"), py::arg("trace") = "",
           py::call_guard<py::gil_scoped_release>())
      .def("wait_completed", &NodeScheduler::wait_completed, py::arg("timeout_s") = 0.0,
           py::call_guard<py::gil_scoped_release>())
      .def("worker_stats",
           [](NodeScheduler& s) {
             std::vector<WorkerStats> ws;
             {
               py::gil_scoped_release rel;
               ws = s.worker_stats();
             }
             py::list out;
             for (const auto& w : ws) {
               py::dict d;
               d["rank"] = w.rank;
               d["ready"] = w.ready;
               d["alive"] = w.alive;
               d["pinned"] = w.pinned;
               d["batches"] = w.batches;
               d["images"] = w.images;
               d["failed_items"] = w.failed_items;
               d["retried_items"] = w.retried_items;
               d["outstanding"] = w.outstanding;
               d["last_hb_age_s"] = w.last_hb_age_s;
               d["gpu_busy_ms"] = w.gpu_busy_ms;
               d["hbm_used"] = w.hbm_used;
               d["hbm_total"] = w.hbm_total;
               d["xgmi_tx_bytes"] = w.xgmi_tx;
               d["xgmi_rx_bytes"] = w.xgmi_rx;
               d["gfx_mhz"] = w.gfx_mhz;
               d["power_w"] = w.power_w;
               d["info"] = w.info;
               out.append(d);
             }
             return out;
           })
      .def("batch_histogram", &NodeScheduler::batch_histogram)
      .def("images_done", &NodeScheduler::images_done)
      .def("open_stat", &NodeScheduler::open_stat)
      .def("stat_counters", &NodeScheduler::stat_counters)
      .def("unlink_stat", &NodeScheduler::unlink_stat)
      .def("set_slot_tags", &NodeScheduler::set_slot_tags, py::arg("name"))
      .def("send_existing", &NodeScheduler::send_existing, py::arg("ids"), py::arg("slots"),
           py::call_guard<py::gil_scoped_release>())
      .def("set_peers", &NodeScheduler::set_peers, py::arg("peers"))
      .def("set_steal", &NodeScheduler::set_steal, py::arg("orphans") = true, py::arg("idle") = true)
      .def("live_workers", &NodeScheduler::live_workers)
      .def("stolen_items", &NodeScheduler::stolen_items)
      .def("stop", &NodeScheduler::stop, py::call_guard<py::gil_scoped_release>());
}
