// tfk-apiserver: single-node Kubernetes-semantics API server (the L0 substrate; no cluster exists here).
#include <cstdio>

#include "../apiserver/server.h"
#include "../operator/options.h"

int main(int argc, char** argv) {
  using namespace tfk;
  std::string host = "127.0.0.1", wal, log_root, level = "info", port_file;
  long long port = 8080, history = 10000;
  bool json = false;
  FlagSet fs("tfk-apiserver");
  fs.add_string("host", &host, "bind address");
  fs.add_int("port", &port, "port (0 = ephemeral)");
  fs.add_string("wal", &wal, "JSON-lines write-ahead log for persistence (optional)");
  fs.add_int("watch-history", &history, "events kept for watch resume (older -> 410 Gone)");
  fs.add_string("port-file", &port_file, "write the bound port here");
  fs.add_bool("json-log-format", &json, "JSON logs");
  fs.add_string("log-level", &level, "log level");
  std::string err;
  if (!fs.parse(argc, argv, &err)) { fprintf(stderr, "%s\n%s", err.c_str(), fs.usage().c_str()); return 2; }
  if (fs.help_requested()) { printf("%s", fs.usage().c_str()); return 0; }
  InitLogging("tfk-apiserver", json, level);
  StopToken stop;
  HandleSignals(stop);
  auto store = std::make_shared<Store>(wal, (size_t)history);
  install_tfjob_crd(*store);
  ApiServer srv(store);
  if (!srv.start(host, (int)port, &err)) { TFK_LOG(Error, "cannot start: " + err); return 1; }
  TFK_LOG(Info, "serving", Json(Json::object_t{{"url", Json("http://" + host + ":" + std::to_string(srv.port()))}}));
  if (!port_file.empty()) {
    FILE* f = fopen(port_file.c_str(), "w");
    if (f) { fprintf(f, "%d\n", srv.port()); fclose(f); }
  }
  printf("listening on http://%s:%d\n", host.c_str(), srv.port());
  fflush(stdout);
  while (!stop.wait_for(1000)) {
  }
  srv.stop();
  return 0;
}
