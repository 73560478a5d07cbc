// tfk-apiserver: single-node Kubernetes-semantics API server (the L0 substrate; no cluster exists here).
#include <cstdio>

#include "../apiserver/server.h"
#include "../operator/options.h"

int main(int argc, char** argv) {
  using namespace tfk;
  std::string host = "127.0.0.1", wal, log_root, level = "info", port_file, tls_cert, tls_key, token_file;
  long long port = 8080, history = 10000, compact = 20000, sync_ms = 100, max_conns = 4096;
  std::string wal_sync = "interval";
  bool json = false;
  FlagSet fs("tfk-apiserver");
  fs.add_string("host", &host, "bind address");
  fs.add_int("port", &port, "port (0 = ephemeral)");
  fs.add_string("wal", &wal, "JSON-lines write-ahead log for persistence (optional)");
  fs.add_int("watch-history", &history, "events kept for watch resume (older -> 410 Gone)");
  fs.add_string("wal-sync", &wal_sync, "WAL fdatasync: always | interval (group commit) | none");
  fs.add_int("wal-sync-interval-ms", &sync_ms, "group-commit interval for --wal-sync=interval");
  fs.add_int("wal-compact-records", &compact, "compact the WAL into a snapshot past this many records (0 = never)");
  fs.add_int("max-connections", &max_conns, "concurrent connections before new ones get 503");
  fs.add_string("port-file", &port_file, "write the bound port here");
  fs.add_bool("json-log-format", &json, "JSON logs");
  fs.add_string("log-level", &level, "log level");
  fs.add_string("tls-cert-file", &tls_cert, "serve HTTPS with this PEM certificate (chain)");
  fs.add_string("tls-private-key-file", &tls_key, "PEM private key for --tls-cert-file");
  fs.add_string("token-auth-file", &token_file, "CSV token,user,uid: require bearer-token authentication");
  std::string err;
  if (!fs.parse(argc, argv, &err)) { fprintf(stderr, "%s\n%s", err.c_str(), fs.usage().c_str()); return 2; }
  if (fs.help_requested()) { printf("%s", fs.usage().c_str()); return 0; }
  InitLogging("tfk-apiserver", json, level);
  StopToken stop;
  HandleSignals(stop);
  if (wal_sync != "always" && wal_sync != "interval" && wal_sync != "none") {
    fprintf(stderr, "--wal-sync must be always|interval|none\n");
    return 2;
  }
  WalOptions wo;
  wo.sync = wal_sync;
  wo.sync_interval_ms = sync_ms;
  wo.compact_records = (size_t)compact;
  auto store = std::make_shared<Store>(wal, (size_t)history, wo);
  install_tfjob_crd(*store);
  ApiServer srv(store);
  if (!tls_cert.empty()) {
    TlsOptions o;
    o.enabled = true;
    o.cert_file = tls_cert;
    o.key_file = tls_key;
    if (!srv.enable_tls(o, &err)) { TFK_LOG(Error, "tls: " + err); return 1; }
  }
  if (!token_file.empty() && !srv.load_token_file(token_file, &err)) { TFK_LOG(Error, err); return 1; }
  srv.set_max_connections((int)max_conns);
  if (!srv.start(host, (int)port, &err)) { TFK_LOG(Error, "cannot start: " + err); return 1; }
  const std::string scheme = srv.tls() ? "https://" : "http://";
  TFK_LOG(Info, "serving", Json(Json::object_t{{"url", Json(scheme + host + ":" + std::to_string(srv.port()))}}));
  if (!port_file.empty()) {
    // write-then-rename: a reader polling for the file never sees it created but still empty
    const std::string tmp = port_file + ".tmp";
    FILE* f = fopen(tmp.c_str(), "w");
    if (f) {
      fprintf(f, "%d\n", srv.port());
      fclose(f);
      std::rename(tmp.c_str(), port_file.c_str());
    }
  }
  printf("listening on %s%s:%d\n", scheme.c_str(), host.c_str(), srv.port());
  fflush(stdout);
  while (!stop.wait_for(1000)) {
  }
  srv.stop();
  return 0;
}
