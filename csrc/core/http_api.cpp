#include "http_api.h"

#include <dirent.h>

#include <chrono>
#include <sstream>

#include "json.h"
#include "pull.h"

namespace zest {

ApiServer::ApiServer(Config& cfg, bt::BtServer* bt, storage::XorbRegistry* registry, std::string self_exe)
    : cfg_(cfg), bt_(bt), registry_(registry), self_exe_(std::move(self_exe)) {
  started_ = std::chrono::steady_clock::now();
  server_ = std::make_unique<http::Server>(net::Addr::loopback(cfg.http_port),
                                           [this](const http::Request& r) { return route(r); }, 8);
}

ApiServer::~ApiServer() {
  stop();
  for (auto& t : job_threads_)
    if (t.joinable()) t.join();
}

void ApiServer::start() { server_->start(); }

void ApiServer::run_until_stopped() {
  start();
  while (!stop_.load()) std::this_thread::sleep_for(std::chrono::milliseconds(50));
  server_->stop();
}

void ApiServer::stop() { stop_.store(true); }

std::string ApiServer::status_json() const {
  bt::ServerStats s = bt_ ? bt_->stats() : bt::ServerStats{};
  json::Writer w;
  w.obj();
  w.key("version").str(kVersion);
  w.key("bt_peers").num_u(s.active_peers);
  w.key("chunks_served").num_u(s.chunks_served);
  w.key("xorbs_cached").num_u(registry_ ? registry_->count() : 0);
  w.key("http_requests").num_u(server_ ? server_->requests() : 0);
  w.key("http_port").num(int64_t(cfg_.http_port));
  w.key("bt_port").num(int64_t(bt_ ? bt_->port() : cfg_.listen_port));
  w.key("bytes_served").num_u(s.bytes_served);
  w.key("total_peers").num_u(s.total_peers);
  w.key("not_found").num_u(s.not_found);
  w.key("rejected").num_u(s.rejected);
  // connection-thread seconds spent finding runs, waiting for device copies and writing sockets
  w.key("serve_lookup_s").num(double(s.lookup_ns) * 1e-9, 4);
  w.key("serve_wait_s").num(double(s.wait_ns) * 1e-9, 4);
  w.key("serve_send_s").num(double(s.send_ns) * 1e-9, 4);
  w.key("uptime_s").num(std::chrono::duration<double>(std::chrono::steady_clock::now() - started_).count(), 1);
  w.key("peer_id").str(std::string(reinterpret_cast<const char*>(cfg_.peer_id.data()), 8));
  if (extra_) w.key("device").raw(extra_());
  w.end();
  return w.out();
}

std::string ApiServer::models_json() const {
  json::Writer w;
  w.arr();
  DIR* d = ::opendir(cfg_.hf_cache_dir.c_str());
  if (d) {
    while (dirent* e = ::readdir(d)) {
      std::string name = e->d_name;
      if (name.rfind("models--", 0) != 0 || name.size() == 8) continue;
      std::string raw = name.substr(8);
      size_t sep = raw.find("--");
      std::string repo = sep == std::string::npos ? raw : raw.substr(0, sep) + "/" + raw.substr(sep + 2);
      size_t files = 0;
      std::string snaps = cfg_.hf_cache_dir + "/" + name + "/snapshots";
      if (DIR* sd = ::opendir(snaps.c_str())) {
        while (dirent* s = ::readdir(sd)) {
          std::string sn = s->d_name;
          if (sn == "." || sn == "..") continue;
          if (DIR* fd = ::opendir((snaps + "/" + sn).c_str())) {
            while (dirent* f = ::readdir(fd)) {
              std::string fn = f->d_name;
              if (fn != "." && fn != "..") ++files;
            }
            ::closedir(fd);
          }
          break;  // first snapshot, like the reference
        }
        ::closedir(sd);
      }
      w.obj().key("name").str(repo).key("files").num(int64_t(files)).end();
    }
    ::closedir(d);
  }
  w.end();
  return w.out();
}

std::shared_ptr<PullJob> ApiServer::start_job(const http::Request& r, int* status, std::string* err) {
  json::Value body;
  try {
    body = r.body.empty() ? json::Value() : json::Value::parse(r.body);
  } catch (const Error&) {
    *status = 400;
    *err = "{\"error\":\"invalid json\"}";
    return nullptr;
  }
  auto job = std::make_shared<PullJob>();
  job->repo = body.str_or("repo", "");
  job->revision = body.str_or("revision", "main");
  if (job->repo.empty()) {
    *status = 400;
    *err = "{\"error\":\"missing repo\"}";
    return nullptr;
  }
  PullOptions opt;
  opt.repo_id = job->repo;
  opt.revision = job->revision;
  opt.p2p = !(body["no_p2p"].type() == json::Value::Type::Bool && body["no_p2p"].as_bool());
  opt.autostart_server = false;
  opt.progress = job->progress;
  for (auto& pe : body["peers"].array())
    if (pe.is_string()) opt.peers.push_back(pe.as_string());
  {
    std::lock_guard<std::mutex> g(jobs_mu_);
    job->id = std::to_string(jobs_.size() + 1);
    jobs_[job->id] = job;
  }
  std::lock_guard<std::mutex> g(jobs_mu_);
  job_threads_.emplace_back([this, job, opt] {
    job->phase = 1;
    std::ostringstream out, err;
    try {
      Config c = cfg_;
      PullSummary s = run_pull(c, opt, out, err);
      {
        std::lock_guard<std::mutex> jg(job->mu);
        job->snapshot = s.snapshot_dir;
        job->stats_json = s.stats_json;
        if (s.failed_files) job->error = std::to_string(s.failed_files) + " file(s) failed";
        job->log = out.str() + err.str();
      }
      if (registry_) registry_->scan(cfg_);
      job->phase = s.failed_files ? 3 : 2;
    } catch (const std::exception& e) {
      {
        std::lock_guard<std::mutex> jg(job->mu);
        job->error = e.what();
        job->log = out.str() + err.str();
      }
      job->phase = 3;
    }
  });
  return job;
}

http::ServerResponse ApiServer::sse(std::shared_ptr<PullJob> job) {
  http::ServerResponse resp;
  resp.content_type = "text/event-stream";
  resp.extra.emplace_back("Cache-Control", "no-cache");
  resp.stream_len = http::ServerResponse::kUntilClose;
  resp.stream = [this, job](net::Socket& s) {
    auto send = [&](const char* ev, const std::string& data) {
      const std::string m = std::string("event: ") + ev + "\ndata: " + data + "\n\n";
      s.write_all(m.data(), m.size());
    };
    PullProgress& pr = *job->progress;
    std::vector<int> seen;
    uint64_t last_bytes = ~uint64_t(0);
    try {
      {
        json::Writer w;
        w.obj().key("job").str(job->id).key("repo").str(job->repo).key("revision").str(job->revision).end();
        send("job", w.out());
      }
      while (true) {
        const int ph = job->phase.load();  // read before the counters: a finished job's are final
        if (pr.listed.load()) {
          std::lock_guard<std::mutex> g(pr.mu);
          seen.resize(pr.files.size(), 0);
          for (size_t i = 0; i < pr.files.size(); ++i) {
            const int st = pr.files[i]->state.load();
            if (st == seen[i]) continue;
            seen[i] = st;
            static const char* names[] = {"queued", "running", "done", "failed", "cached"};
            json::Writer w;
            w.obj().key("path").str(pr.files[i]->path).key("size").num_u(pr.files[i]->size);
            w.key("index").num(int64_t(i + 1)).key("total").num(int64_t(pr.files.size()));
            w.key("state").str(names[st]).end();
            send("file", w.out());
          }
        }
        const uint64_t b = pr.bytes.load();
        if (b != last_bytes && pr.listed.load()) {
          last_bytes = b;
          json::Writer w;
          w.obj().key("bytes").num_u(b).key("total").num_u(pr.total.load());
          w.key("source").str(PullProgress::source_name(pr.last_source.load()));
          w.key("peers").num_u(pr.peers.load()).key("from_peer").num_u(pr.from_peer.load());
          w.key("from_cdn").num_u(pr.from_cdn.load()).key("from_cache").num_u(pr.from_cache.load()).end();
          send("progress", w.out());
        }
        if (ph >= 2) {
          json::Writer w;
          std::lock_guard<std::mutex> g(job->mu);
          if (ph == 2) {
            w.obj().key("path").str(job->snapshot).key("stats").raw(job->stats_json).end();
            send("complete", w.out());
          } else {
            w.obj().key("error").str(job->error).key("path").str(job->snapshot).end();
            send("error", w.out());
          }
          return;
        }
        if (stop_.load()) return;
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
      }
    } catch (const Error&) {  // client went away
    }
  };
  return resp;
}

http::ServerResponse ApiServer::route(const http::Request& r) {
  http::ServerResponse resp;
  const std::string& p = r.path;
  if (p == "/v1/health") {
    resp.body = "{\"status\":\"ok\"}";
  } else if (p == "/v1/status") {
    resp.body = status_json();
  } else if (p == "/v1/stop") {
    resp.body = "{\"status\":\"shutting down\"}";
    stop();
    if (bt_) std::thread([bt = bt_] { bt->stop(); }).detach();
  } else if (p == "/v1/models") {
    resp.body = models_json();
  } else if (p == "/v1/config") {
    resp.body = cfg_.to_json();
  } else if (p == "/v1/pull" && r.method == "POST") {
    int status = 200;
    std::string err;
    auto job = start_job(r, &status, &err);
    if (!job) {
      resp.status = status;
      resp.body = err;
      return resp;
    }
    auto it = r.query.find("stream");
    if (r.header("accept").find("text/event-stream") != std::string::npos || (it != r.query.end() && it->second == "1"))
      return sse(job);
    resp.body = "{\"status\":\"started\",\"job\":\"" + job->id + "\"}";
  } else if (p.rfind("/v1/pull/", 0) == 0) {
    std::string id = p.substr(9);
    const bool events = id.size() > 7 && id.compare(id.size() - 7, 7, "/events") == 0;
    if (events) id.resize(id.size() - 7);
    std::shared_ptr<PullJob> job;
    {
      std::lock_guard<std::mutex> g(jobs_mu_);
      auto it = jobs_.find(id);
      if (it != jobs_.end()) job = it->second;
    }
    if (!job) {
      resp.status = 404;
      resp.body = "{\"error\":\"no such pull job\"}";
    } else if (events) {
      return sse(job);
    } else {
      const PullProgress& pr = *job->progress;
      const uint64_t bytes = pr.bytes.load(), total = pr.total.load();
      const int ph = job->phase.load();
      json::Writer w;
      std::lock_guard<std::mutex> g(job->mu);
      w.obj().key("job").str(job->id).key("repo").str(job->repo).key("revision").str(job->revision);
      w.key("state").str(job->state());
      w.key("progress").num(ph == 2 ? 1.0 : total ? double(bytes) / double(total) : 0.0, 4);
      w.key("bytes").num_u(bytes).key("total").num_u(total);
      w.key("from_peer").num_u(pr.from_peer.load()).key("from_cdn").num_u(pr.from_cdn.load());
      w.key("from_cache").num_u(pr.from_cache.load()).key("peers").num_u(pr.peers.load());
      w.key("snapshot").str(job->snapshot).key("error").str(job->error).key("stats").raw(job->stats_json);
      w.key("log").str(job->log).end();
      resp.body = w.out();
    }
  } else if (p == "/metrics") {
    bt::ServerStats s = bt_ ? bt_->stats() : bt::ServerStats{};
    std::ostringstream m;
    m << "# TYPE zest_chunks_served_total counter\nzest_chunks_served_total " << s.chunks_served << "\n";
    m << "# TYPE zest_bytes_served_total counter\nzest_bytes_served_total " << s.bytes_served << "\n";
    m << "# TYPE zest_bt_peers gauge\nzest_bt_peers " << s.active_peers << "\n";
    m << "# TYPE zest_bt_peers_total counter\nzest_bt_peers_total " << s.total_peers << "\n";
    m << "# TYPE zest_bt_rejected_total counter\nzest_bt_rejected_total " << s.rejected << "\n";
    m << "# TYPE zest_chunk_not_found_total counter\nzest_chunk_not_found_total " << s.not_found << "\n";
    m << "# TYPE zest_xorbs_cached gauge\nzest_xorbs_cached " << (registry_ ? registry_->count() : 0) << "\n";
    m << "# TYPE zest_http_requests_total counter\nzest_http_requests_total " << server_->requests() << "\n";
    resp.content_type = "text/plain; version=0.0.4";
    resp.body = m.str();
  } else if (p == "/" || p == "/ui") {
    resp.content_type = "text/html; charset=utf-8";
    resp.body = kDashboardHtml;
  } else {
    resp.status = 404;
    resp.body = "{\"error\":\"not found\"}";
  }
  return resp;
}

const char* kDashboardHtml = R"HTML(<!doctype html>
<html><head><meta charset="utf-8"><title>zest (MI355X)</title>
<style>
body{font:14px system-ui,sans-serif;background:#0f1115;color:#e6e6e6;margin:2rem}
h1{font-size:20px} .grid{display:grid;grid-template-columns:repeat(auto-fill,minmax(180px,1fr));gap:12px}
.card{background:#1a1d24;border-radius:8px;padding:12px}.k{color:#8a93a6;font-size:12px}.v{font-size:22px}
table{border-collapse:collapse;margin-top:1rem;width:100%}td,th{border-bottom:1px solid #2a2f3a;padding:6px;text-align:left}
button{background:#c0392b;color:#fff;border:0;border-radius:6px;padding:6px 14px;cursor:pointer}
</style></head><body>
<h1>zest &mdash; P2P model distribution on AMD Instinct</h1>
<div class="grid" id="cards"></div>
<table><thead><tr><th>model</th><th>files</th></tr></thead><tbody id="models"></tbody></table>
<p><button onclick="fetch('/v1/stop',{method:'POST'}).then(()=>document.title='stopped')">Stop server</button></p>
<script>
const keys=["version","bt_peers","chunks_served","bytes_served","xorbs_cached","http_requests","bt_port","uptime_s"];
async function tick(){
 try{const s=await (await fetch('/v1/status')).json();
  document.getElementById('cards').innerHTML=keys.map(k=>`<div class="card"><div class="k">${k}</div><div class="v">${s[k]}</div></div>`).join('');
  const m=await (await fetch('/v1/models')).json();
  document.getElementById('models').innerHTML=m.map(x=>`<tr><td>${x.name}</td><td>${x.files}</td></tr>`).join('');
 }catch(e){}
}
tick();setInterval(tick,2000);
</script></body></html>)HTML";

}  // namespace zest
