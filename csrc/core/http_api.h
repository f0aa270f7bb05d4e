// Local REST API + dashboard for `zest serve` (loopback only).
//
// Reference: src/http_api.zig:1-375 — binds 127.0.0.1:http_port (:49); routes /v1/health,
// /v1/status {"version","bt_peers","chunks_served","xorbs_cached","http_requests","http_port",
// "bt_port"} (:120-136), /v1/stop (:144-149), /v1/pull* (a stub there, :138-142), /v1/models
// (:152-210), / and /ui dashboard (:212-221, :235-351), 404 {"error":"not found"}.
// Here /v1/pull really pulls (POST {"repo","revision",...} -> background job, GET /v1/pull/{id}
// for byte progress; with `Accept: text/event-stream` (or ?stream=1) the POST answers with the
// job's SSE stream as DESIGN.md:317-338 specifies, and GET /v1/pull/{id}/events streams an
// existing job), the server is multi-threaded, xorb counts are live, and /metrics exports
// Prometheus counters.  Keys of the reference's status JSON are kept; GPU/seeding fields are added.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "bt_server.h"
#include "config.h"
#include "http.h"
#include "pull.h"
#include "storage.h"

namespace zest {

struct PullJob {
  std::string id, repo, revision, error, snapshot;
  std::atomic<int> phase{0};  // 0 queued, 1 running, 2 done, 3 error (strings via state())
  std::string log;
  std::string stats_json = "{}";
  std::shared_ptr<PullProgress> progress = std::make_shared<PullProgress>();
  std::mutex mu;  // guards the strings written when the job ends
  const char* state() const {
    static const char* names[] = {"queued", "running", "done", "error"};
    return names[phase.load()];
  }
};

class ApiServer {
 public:
  ApiServer(Config& cfg, bt::BtServer* bt, storage::XorbRegistry* registry, std::string self_exe);
  ~ApiServer();
  void start();
  void run_until_stopped();
  void stop();
  bool stopping() const { return stop_.load(); }
  uint16_t port() const { return server_ ? server_->port() : 0; }
  // Extra status fields (e.g. HBM cache from the Python layer).
  void set_extra_status(std::function<std::string()> f) { extra_ = std::move(f); }

 private:
  http::ServerResponse route(const http::Request& r);
  // Server-Sent Events of one pull job: `file` (a file started or finished), `progress` (bytes,
  // total, source, peers; at most every 200 ms while bytes move) and a final `complete` / `error`.
  http::ServerResponse sse(std::shared_ptr<PullJob> job);
  std::shared_ptr<PullJob> start_job(const http::Request& r, int* status, std::string* err);
  std::string status_json() const;
  std::string models_json() const;
  Config& cfg_;
  bt::BtServer* bt_;
  storage::XorbRegistry* registry_;
  std::string self_exe_;
  std::unique_ptr<http::Server> server_;
  std::atomic<bool> stop_{false};
  std::mutex jobs_mu_;
  std::map<std::string, std::shared_ptr<PullJob>> jobs_;
  std::vector<std::thread> job_threads_;
  std::function<std::string()> extra_;
  std::chrono::steady_clock::time_point started_;
};

extern const char* kDashboardHtml;

}  // namespace zest
