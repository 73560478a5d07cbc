// tfk-unit-tests: control-plane unit tests (the reference ships none -- its
// upstream tree names defaults_test.go, validation_test.go, helpers_test.go, training_test.go,
// replicas_test.go: images/tf3.PNG:L8-L17). Run: build/bin/tfk-unit-tests [filter]
// Exit status 0 only if every selected test passes. Also built under TSan/ASan (make SAN=...).
#include <unistd.h>
#include <sys/socket.h>
#include <netinet/in.h>
#include <arpa/inet.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../api/types.h"
#include "../apiserver/server.h"
#include "../apiserver/store.h"
#include "../cache/informer.h"
#include "../client/client.h"
#include "../kubelet/probe.h"
#include "../common/json.h"
#include "../common/util.h"
#include "../controller/trainer.h"
#include "../kubelet/kubelet.h"
#include "../leaderelection/leaderelection.h"
#include "../runtime/tfbundle.h"
#include "../scheduler/scheduler.h"
#include "../util/workqueue.h"
#include "testing.h"

using namespace tfk;

namespace {
Json J(const std::string& s) { return Json::parse(s); }

std::shared_ptr<Store> new_store() {
  auto s = std::make_shared<Store>();
  install_tfjob_crd(*s);
  return s;
}

Json container(const std::string& name = "tensorflow") {
  return J(R"({"name":")" + name + R"(","image":"tfk/runtime","command":["python3","-c","pass"]})");
}

Json v1_job(const std::string& name, int workers, int ps = 0, bool chief = true) {
  Json job = J(R"({"apiVersion":"kubeflow.org/v1","kind":"TFJob","metadata":{"name":"","namespace":"default"},
                    "spec":{"tfReplicaSpecs":{}}})");
  job["metadata"]["name"] = name;
  auto rs = [&](int n) {
    Json r = Json::object();
    r["replicas"] = n;
    r["restartPolicy"] = "ExitCode";
    r["template"]["spec"]["containers"] = Json::array();
    r["template"]["spec"]["containers"].push_back(container());
    return r;
  };
  if (chief) job["spec"]["tfReplicaSpecs"]["Chief"] = rs(1);
  if (workers) job["spec"]["tfReplicaSpecs"]["Worker"] = rs(workers);
  if (ps) job["spec"]["tfReplicaSpecs"]["PS"] = rs(ps);
  return job;
}
}  // namespace

// ----------------------------------------------------------------------------- JSON / util
TEST(json_roundtrip) {
  Json j = J(R"({"a":[1,2.5,"x",true,null],"b":{"c":"é\n"}})");
  CHECK_EQ(j.path("b.c").str(), std::string("\xc3\xa9\n"));
  CHECK(Json::parse(j.dump()) == j);
  CHECK_EQ(j.at("a")[1].as_double(), 2.5);
  CHECK(j.at("missing").is_null());
  bool threw = false;
  try {
    Json::parse("{\"a\":");
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
}

TEST(crc32c_known_vector) {
  // RFC 3720 B.4: crc32c("123456789") = 0xE3069283
  CHECK_EQ(crc32c("123456789", 9), 0xE3069283u);
  CHECK_EQ(crc32c_unmask(crc32c_mask(0xdeadbeefu)), 0xdeadbeefu);
}

// ----------------------------------------------------------------------------- API types
TEST(defaults_v1alpha1) {
  api::TFJob job = api::from_json(J(R"({"apiVersion":"kubeflow.org/v1alpha1","kind":"TFJob",
      "metadata":{"name":"j","namespace":"default"},
      "spec":{"replicaSpecs":[{"template":{"spec":{"containers":[{"name":"tensorflow","image":"x"}]}}},
                              {"tfReplicaType":"WORKER","replicas":3,
                               "template":{"spec":{"containers":[{"name":"tensorflow","image":"x"}]}}}]}})"));
  api::set_defaults(job);
  const api::ReplicaSpec* m = job.replica(api::RType::Master);
  CHECK(m != nullptr);
  CHECK_EQ(m->replicas, 1);
  CHECK_EQ(m->tf_port, 2222);
  CHECK_EQ(job.replica(api::RType::Worker)->replicas, 3);
  CHECK_EQ(job.chief_name, std::string("MASTER"));
  CHECK_EQ(job.chief_index, 0);
  CHECK(api::validate(job).empty());
}

TEST(validation_errors) {
  // no container named tensorflow
  api::TFJob a = api::from_json(J(R"({"apiVersion":"kubeflow.org/v1","kind":"TFJob","metadata":{"name":"j"},
      "spec":{"tfReplicaSpecs":{"Worker":{"replicas":1,"template":{"spec":{"containers":[{"name":"main"}]}}}}}})"));
  api::set_defaults(a);
  CHECK(!api::validate(a).empty());
  // two chiefs
  Json jb = v1_job("b", 1);
  jb["spec"]["tfReplicaSpecs"]["Chief"]["replicas"] = 2;
  api::TFJob b = api::from_json(jb);
  api::set_defaults(b);
  CHECK(!api::validate(b).empty());
  // a good one
  api::TFJob c = api::from_json(v1_job("c", 2, 1));
  api::set_defaults(c);
  CHECK(api::validate(c).empty());
}

TEST(version_conversion_roundtrip) {
  Json v1 = v1_job("conv", 2, 1);
  Json a1 = api::convert(v1, "kubeflow.org/v1alpha1");
  CHECK_EQ(a1.at("apiVersion").str(), std::string("kubeflow.org/v1alpha1"));
  CHECK(a1.path("spec.replicaSpecs").is_array());
  Json back = api::convert(a1, "kubeflow.org/v1");
  CHECK_EQ(back.path("spec.tfReplicaSpecs.Worker.replicas").as_int(), 2LL);
  CHECK_EQ(back.path("spec.tfReplicaSpecs.PS.replicas").as_int(), 1LL);
}

TEST(v1alpha1_only_fields_survive_v1_storage) {
  Json a = J(R"({"apiVersion":"kubeflow.org/v1alpha1","kind":"TFJob","metadata":{"name":"x","namespace":"default"},
      "spec":{"runtimeId":"ab12","tfImage":"tf:1.5","terminationPolicy":{"chief":{"replicaName":"WORKER","replicaIndex":1}},
              "replicaSpecs":[{"replicas":2,"tfReplicaType":"WORKER","template":{"spec":{"containers":[{"name":"tensorflow"}]}}}]}})");
  Json v1 = api::convert(a, "kubeflow.org/v1");
  CHECK_EQ(v1.path("metadata.annotations").at(api::kAnnRuntimeId).str(), std::string("ab12"));
  Json back = api::convert(v1, "kubeflow.org/v1alpha1");
  CHECK_EQ(back.path("spec.runtimeId").str(), std::string("ab12"));
  CHECK_EQ(back.path("spec.tfImage").str(), std::string("tf:1.5"));
  CHECK_EQ(back.path("spec.terminationPolicy.chief.replicaName").str(), std::string("WORKER"));
  CHECK_EQ(back.path("spec.terminationPolicy.chief.replicaIndex").as_int(), 1LL);
  CHECK(!back.path("metadata.annotations").is_object() || !back.path("metadata.annotations").has(api::kAnnRuntimeId));
}

TEST(gen_name_and_tf_config) {
  api::TFJob job = api::from_json(v1_job(std::string(50, 'x'), 2, 1));
  api::set_defaults(job);
  std::string n = api::gen_name(job, api::RType::Worker, 1);
  CHECK(n.size() <= 63);
  CHECK(n.find("worker-1") != std::string::npos);
  Json tf = Json::parse(api::tf_config(job, api::RType::Worker, 1, ""));
  CHECK_EQ(tf.path("task.type").str(), std::string("worker"));
  CHECK_EQ(tf.path("task.index").as_int(), 1LL);
  CHECK_EQ(tf.path("cluster.worker").size(), (size_t)2);
  CHECK_EQ(tf.path("cluster.ps").size(), (size_t)1);
  CHECK_EQ(tf.path("cluster.chief").size(), (size_t)1);
  CHECK(tf.path("cluster.worker")[0].str().find(":2222") != std::string::npos);
  CHECK_EQ(tf.at("environment").str(), std::string("cloud"));
}

TEST(evaluator_not_in_cluster_spec) {
  Json j = v1_job("ev", 1);
  Json ev = j.path("spec.tfReplicaSpecs.Worker").clone();
  ev["replicas"] = 1;
  j["spec"]["tfReplicaSpecs"]["Evaluator"] = ev;
  api::TFJob job = api::from_json(j);
  api::set_defaults(job);
  Json tf = Json::parse(api::tf_config(job, api::RType::Evaluator, 0, ""));
  CHECK(!tf.at("cluster").has("evaluator"));
  CHECK_EQ(tf.path("task.type").str(), std::string("evaluator"));
}

TEST(retryable_exit_codes) {
  CHECK(!api::is_retryable_exit(1, ""));
  CHECK(!api::is_retryable_exit(127, ""));
  CHECK(api::is_retryable_exit(137, ""));
  CHECK(api::is_retryable_exit(143, ""));
  CHECK(!api::is_retryable_exit(137, "OOMKilled"));
}

TEST(accelerator_injection) {
  Json j = v1_job("gpu", 1, 0, false);
  j["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][(size_t)0]["resources"]["limits"]["amd.com/gpu"] = 1;
  api::TFJob job = api::from_json(j);
  api::set_defaults(job);
  api::configure_accelerators(job, api::ControllerConfig::defaults());
  std::string dumped = api::to_json(job).dump();
  CHECK(dumped.find("/dev/kfd") != std::string::npos);
  CHECK(dumped.find("/dev/dri") != std::string::npos);
}

// ----------------------------------------------------------------------------- store semantics
TEST(store_rv_conflict_and_status) {
  auto s = new_store();
  Json out;
  CHECK(s->create("pods", "default", J(R"({"metadata":{"name":"p"},"spec":{}})"), &out).ok());
  Json stale = out.clone();
  out["spec"]["x"] = 1;
  Json out2;
  CHECK(s->update("pods", "default", "p", out, false, &out2).ok());
  CHECK(out2.path("metadata.resourceVersion").str() != stale.path("metadata.resourceVersion").str());
  stale["spec"]["y"] = 2;
  CHECK_EQ(s->update("pods", "default", "p", stale, false, &out).code, 409);
  CHECK_EQ(s->create("pods", "default", J(R"({"metadata":{"name":"p"}})"), &out).code, 409);
  // status subresource only changes status
  Json st = out2.clone();
  st["status"]["phase"] = "Running";
  st["spec"]["x"] = 99;
  CHECK(s->update("pods", "default", "p", st, true, &out).ok());
  CHECK_EQ(out.path("status.phase").str(), std::string("Running"));
  CHECK_EQ(out.path("spec.x").as_int(), 1LL);
}

TEST(store_finalizers_and_gc) {
  auto s = new_store();
  Json owner;
  CHECK(s->create("tfjobs", "default", J(R"({"apiVersion":"kubeflow.org/v1","kind":"TFJob","metadata":{"name":"o",
      "finalizers":["tfjob.kubeflow.org/cleanup"]},"spec":{"tfReplicaSpecs":{}}})"), &owner).ok());
  Json pod = J(R"({"metadata":{"name":"child","ownerReferences":[{"apiVersion":"kubeflow.org/v1","kind":"TFJob",
      "name":"o","controller":true}]}})");
  pod["metadata"]["ownerReferences"][(size_t)0]["uid"] = owner.path("metadata.uid");
  Json out;
  CHECK(s->create("pods", "default", pod, &out).ok());
  CHECK(s->remove("tfjobs", "default", "o", "Background", &out).ok());
  // finalizer keeps the object, with a deletionTimestamp
  CHECK(s->get("tfjobs", "default", "o", &out).ok());
  CHECK(!out.path("metadata.deletionTimestamp").is_null());
  // removing the finalizer completes the delete and garbage-collects the dependent
  out["metadata"]["finalizers"] = Json::array();
  Json o2;
  CHECK(s->update("tfjobs", "default", "o", out, false, &o2).ok());
  CHECK_EQ(s->get("tfjobs", "default", "o", &out).code, 404);
  CHECK_EQ(s->get("pods", "default", "child", &out).code, 404);
}

// a dependent that cascade GC marks terminating (it has finalizers) must keep that
// state across an apiserver restart (WAL replay).
TEST(store_gc_terminating_dependent_survives_wal_replay) {
  char tmpl[] = "/tmp/tfk-wal-XXXXXX";
  int fd = mkstemp(tmpl);
  CHECK(fd >= 0);
  close(fd);
  std::string path = tmpl;
  {
    Store s(path);
    install_tfjob_crd(s);
    Json owner, out;
    CHECK(s.create("tfjobs", "default", J(R"({"apiVersion":"kubeflow.org/v1","kind":"TFJob","metadata":{"name":"o"},
        "spec":{"tfReplicaSpecs":{}}})"), &owner).ok());
    Json pod = J(R"({"metadata":{"name":"child","finalizers":["tfk.io/keep"],"ownerReferences":[{"apiVersion":
        "kubeflow.org/v1","kind":"TFJob","name":"o","controller":true}]}})");
    pod["metadata"]["ownerReferences"][(size_t)0]["uid"] = owner.path("metadata.uid");
    CHECK(s.create("pods", "default", pod, &out).ok());
    CHECK(s.remove("tfjobs", "default", "o", "Background", &out).ok());
    CHECK(s.get("pods", "default", "child", &out).ok());
    CHECK(!out.path("metadata.deletionTimestamp").is_null());
  }
  Store s2(path);  // restart: replay the WAL
  Json out;
  CHECK(s2.get("pods", "default", "child", &out).ok());
  CHECK(!out.path("metadata.deletionTimestamp").is_null());
  unlink(path.c_str());
}

TEST(wal_compaction_snapshot_replays_identically) {
  char tmpl[] = "/tmp/tfk-wal-XXXXXX";
  std::string dir = mkdtemp(tmpl);
  std::string wal = dir + "/wal.jsonl";
  WalOptions wo;
  wo.sync = "always";
  wo.compact_records = 40;
  int64_t rv_before = 0;
  {
    Store st(wal, 1000, wo);
    Json out;
    for (int i = 0; i < 5; ++i) {
      Json cm = J(R"({"apiVersion":"v1","kind":"ConfigMap","metadata":{"name":""},"data":{"v":"0"}})");
      cm["metadata"]["name"] = "cm" + std::to_string(i);
      CHECK(st.create("configmaps", "default", cm, &out).ok());
    }
    for (int r = 0; r < 60; ++r) {  // 300 updates of 5 live objects -> several compactions
      for (int i = 0; i < 5; ++i) {
        Json cur;
        CHECK(st.get("configmaps", "default", "cm" + std::to_string(i), &cur).ok());
        cur["data"]["v"] = std::to_string(r);
        CHECK(st.update("configmaps", "default", "cm" + std::to_string(i), cur, false, &out).ok());
      }
    }
    CHECK(st.remove("configmaps", "default", "cm4", "Background", &out).ok());
    rv_before = st.resource_version();
    CHECK(st.counters()["wal_compactions"] > 0);
    CHECK(st.counters()["wal_fsync"] > 300);
  }
  size_t lines = 0;
  {
    FILE* f = fopen(wal.c_str(), "r");
    char buf[65536];
    while (fgets(buf, sizeof buf, f)) lines++;
    fclose(f);
  }
  CHECK(lines < 80);  // compacted: snapshot + the tail since the last compaction, not 306 records
  Store st2(wal, 1000, wo);
  Json cur;
  CHECK(st2.get("configmaps", "default", "cm2", &cur).ok());
  CHECK_EQ(cur.path("data.v").str(), std::string("59"));
  CHECK(!st2.get("configmaps", "default", "cm4", &cur).ok());
  CHECK(st2.resource_version() >= rv_before);  // deleted objects' versions are never reissued
  unlink(wal.c_str());
  rmdir(dir.c_str());
}

TEST(slow_watcher_is_dropped_others_unaffected) {
  auto store = new_store();
  ApiStatus st;
  auto slow = store->watch("configmaps", "default", 0, LabelSelector(), FieldSelector(), &st);
  auto fast = store->watch("configmaps", "default", 0, LabelSelector(), FieldSelector(), &st);
  slow->max_queue_for_test(16);
  Json out;
  int seen = 0;
  for (int i = 0; i < 40; ++i) {
    Json cm = J(R"({"apiVersion":"v1","kind":"ConfigMap","metadata":{"name":""}})");
    cm["metadata"]["name"] = "c" + std::to_string(i);
    CHECK(store->create("configmaps", "default", cm, &out).ok());
    WatchEvent ev;
    while (fast->next(&ev, 0)) seen++;  // the fast consumer keeps up
  }
  CHECK(slow->closed());  // over its queue bound: terminated, the client relists
  WatchEvent ev;
  CHECK(!slow->next(&ev, 0));
  CHECK(!fast->closed());
  CHECK_EQ(seen, 40);
}

TEST(http_server_sheds_connections_over_the_cap) {
  auto store = new_store();
  ApiServer srv(store);
  srv.set_max_connections(2);
  std::string err;
  CHECK(srv.start("127.0.0.1", 0, &err));
  std::vector<int> held;
  for (int i = 0; i < 2; ++i) {  // two idle keep-alive connections occupy the cap
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)srv.port());
    inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
    CHECK(connect(fd, (sockaddr*)&a, sizeof a) == 0);
    held.push_back(fd);
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)srv.port());
  inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
  CHECK(connect(fd, (sockaddr*)&a, sizeof a) == 0);
  char buf[256] = {0};
  ssize_t n = recv(fd, buf, sizeof buf - 1, 0);
  CHECK(n > 0 && std::string(buf).find("503") != std::string::npos);
  ::close(fd);
  // the server counts the shed connection after writing the 503 the client already read
  for (int i = 0; i < 200 && srv.connections_rejected() < 1; ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  CHECK(srv.connections_rejected() >= 1);
  for (int h : held) ::close(h);
  srv.stop();
}

TEST(http_server_stop_returns_with_a_stalled_stream_client) {
  // A watch-style handler streams to a client that stops reading: its send() blocks once the
  // socket buffers fill. stop() must still return promptly (shutdown of live sockets
  // plus SO_SNDTIMEO on accepted connections).
  HttpServer srv;
  std::string err;
  CHECK(srv.listen("127.0.0.1", 0, &err));
  srv.serve([](const HttpRequest&, ResponseWriter& w) {
    w.start_stream(200, "application/json");
    std::string chunk(64 << 10, 'x');
    while (w.alive() && w.write_chunk(chunk)) {
    }
  });
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  int small = 4096;
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &small, sizeof small);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)srv.port());
  inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
  CHECK(connect(fd, (sockaddr*)&a, sizeof a) == 0);
  std::string req = "GET /watch HTTP/1.1\r\nHost: x\r\n\r\n";
  CHECK(send(fd, req.data(), req.size(), 0) == (ssize_t)req.size());
  std::this_thread::sleep_for(std::chrono::milliseconds(500));  // buffers full, handler blocked in send
  CHECK_EQ(srv.connections_active(), 1);
  auto t0 = std::chrono::steady_clock::now();
  srv.stop();
  double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  CHECK(s < 5.0);
  CHECK_EQ(srv.connections_active(), 0);
  ::close(fd);
}

TEST(store_watch_replay_and_gone) {
  auto s = std::make_shared<Store>("", 4);  // tiny history window
  Json out;
  CHECK(s->create("pods", "default", J(R"({"metadata":{"name":"a","labels":{"app":"x"}}})"), &out).ok());
  int64_t rv0 = std::stoll(out.path("metadata.resourceVersion").str());
  CHECK(s->create("pods", "default", J(R"({"metadata":{"name":"b","labels":{"app":"y"}}})"), &out).ok());
  ApiStatus st;
  auto w = s->watch("pods", "default", rv0, LabelSelector::parse("app=y"), FieldSelector(), &st);
  CHECK(st.ok());
  WatchEvent ev;
  CHECK(w->next(&ev, 1000));
  CHECK_EQ(ev.type, std::string("ADDED"));
  CHECK_EQ(ev.object.path("metadata.name").str(), std::string("b"));
  for (int i = 0; i < 10; ++i) {
    Json o;
    s->create("pods", "default", J("{\"metadata\":{\"name\":\"c" + std::to_string(i) + "\"}}"), &o);
  }
  ApiStatus st2;
  auto w2 = s->watch("pods", "default", rv0, LabelSelector(), FieldSelector(), &st2);
  CHECK_EQ(st2.code, 410);
}

TEST(label_and_field_selectors) {
  LabelSelector ls = LabelSelector::parse("a=1,b!=2,c,!d,e in (x,y),f notin (z)");
  CHECK(ls.matches(J(R"({"a":"1","b":"3","c":"","e":"y","f":"q"})")));
  CHECK(!ls.matches(J(R"({"a":"1","b":"2","c":"","e":"y"})")));
  CHECK(!ls.matches(J(R"({"a":"1","c":"","d":"","e":"y"})")));
  FieldSelector fs = FieldSelector::parse("metadata.name=x,status.phase!=Failed");
  CHECK(fs.matches(J(R"({"metadata":{"name":"x"},"status":{"phase":"Running"}})")));
  CHECK(!fs.matches(J(R"({"metadata":{"name":"x"},"status":{"phase":"Failed"}})")));
}

TEST(merge_patch_rfc7386) {
  Json t = J(R"({"a":"b","c":{"d":"e","f":"g"}})");
  Json r = merge_patch(t, J(R"({"a":"z","c":{"f":null}})"));
  CHECK(r == J(R"({"a":"z","c":{"d":"e"}})"));
}

// ----------------------------------------------------------------------------- client / cache / queue
TEST(fake_client_records_actions) {
  auto fc = std::make_shared<FakeClient>(new_store());
  Json out;
  CHECK(fc->create("pods", "default", J(R"({"metadata":{"name":"p1"}})"), &out).ok());
  CHECK(fc->get("pods", "default", "p1", &out).ok());
  CHECK(fc->remove("pods", "default", "p1", "Background").ok());
  auto a = fc->actions();
  CHECK_EQ(a.size(), (size_t)3);
  CHECK(a[0].find("create") == 0);
  CHECK(a[2].find("delete") == 0);
}

TEST(token_bucket_rate) {
  TokenBucket tb(100, 5);
  int ok = 0;
  for (int i = 0; i < 20; ++i) ok += tb.try_accept();
  CHECK(ok >= 5 && ok <= 7);  // burst, maybe one refill
}

TEST(workqueue_dedup_and_processing) {
  RateLimitingQueue q("t");
  q.add("a");
  q.add("a");
  q.add("b");
  CHECK_EQ(q.len(), (size_t)2);
  std::string it;
  CHECK(q.get(&it));
  CHECK_EQ(it, std::string("a"));
  q.add("a");  // while processing -> parked dirty, not queued twice
  CHECK_EQ(q.len(), (size_t)1);
  q.done("a");  // re-queued by done
  CHECK_EQ(q.len(), (size_t)2);
  q.shutdown();
}

TEST(workqueue_rate_limited_backoff) {
  ItemExponentialFailureRateLimiter rl(5, 1000);
  CHECK_EQ(rl.when_ms("x"), (int64_t)5);
  CHECK_EQ(rl.when_ms("x"), (int64_t)10);
  CHECK_EQ(rl.when_ms("x"), (int64_t)20);
  CHECK_EQ(rl.num_requeues("x"), 3);
  rl.forget("x");
  CHECK_EQ(rl.when_ms("x"), (int64_t)5);
  for (int i = 0; i < 20; ++i) rl.when_ms("y");
  CHECK_EQ(rl.when_ms("y"), (int64_t)1000);
  RateLimitingQueue q("t2");
  auto t0 = mono_ms();
  q.add_after("z", 50);
  std::string it;
  CHECK(q.get(&it));
  CHECK(mono_ms() - t0 >= 45);
  q.shutdown();
}

TEST(informer_sync_and_events) {
  auto store = new_store();
  auto fc = std::make_shared<FakeClient>(store);
  Json out;
  fc->create("pods", "default", J(R"({"metadata":{"name":"p0"}})"), &out);
  StopToken stop;  // must outlive the informer's threads (declared first, destroyed last)
  SharedInformer inf(fc, "pods", "", 0);
  std::atomic<int> adds{0}, updates{0}, deletes{0};
  inf.add_event_handler({[&](const Json&) { adds++; }, [&](const Json&, const Json&) { updates++; },
                         [&](const Json&) { deletes++; }});
  inf.start(stop);
  CHECK(inf.wait_for_sync(5000));
  fc->create("pods", "default", J(R"({"metadata":{"name":"p1"}})"), &out);
  out["spec"]["x"] = 1;
  Json o2;
  fc->update("pods", "default", out, &o2);
  fc->remove("pods", "default", "p0", "Background");
  auto dl = mono_ms() + 5000;
  while (mono_ms() < dl && !(adds >= 2 && updates >= 1 && deletes >= 1)) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  stop.stop();
  CHECK(adds >= 2);
  CHECK(updates >= 1);
  CHECK(deletes >= 1);
  Lister l(inf.indexer());
  CHECK(l.get("default", "p1", &out));
  CHECK(!l.get("default", "p0", &out));
}

TEST(leader_election_single_holder) {
  auto store = new_store();
  auto c = std::make_shared<FakeClient>(store);
  LeaderElectionConfig a, b;
  a.identity = "a";
  b.identity = "b";
  a.lease_duration_ms = b.lease_duration_ms = 300;
  LeaderElector ea(c, a), eb(c, b);
  CHECK(ea.try_acquire_or_renew());
  CHECK(!eb.try_acquire_or_renew());
  CHECK_EQ(eb.observed_leader(), std::string("a"));
  std::this_thread::sleep_for(std::chrono::milliseconds(400));  // lease expires
  CHECK(eb.try_acquire_or_renew());
  CHECK(!ea.try_acquire_or_renew());
}

// ----------------------------------------------------------------------------- scheduler
TEST(gang_placement_all_or_nothing) {
  auto pod = [](const std::string& n, int g) {
    Json p = J(R"({"metadata":{"name":""},"spec":{"containers":[{"name":"tensorflow","resources":{"limits":{}}}]}})");
    p["metadata"]["name"] = n;
    p["spec"]["containers"][(size_t)0]["resources"]["limits"]["amd.com/gpu"] = g;
    return p;
  };
  std::vector<NodeInfo> nodes(1);
  nodes[0].name = "n0";
  nodes[0].gpus = 8;
  std::vector<Json> group;
  for (int i = 0; i < 8; ++i) group.push_back(pod("w" + std::to_string(i), 1));
  auto pl = GangScheduler::place_group(group, nodes);
  CHECK_EQ(pl.size(), (size_t)8);
  std::set<int> ids;
  for (auto& kv : pl)
    for (int g : kv.second.second) ids.insert(g);
  CHECK_EQ(ids.size(), (size_t)8);  // disjoint GPUs
  group.push_back(pod("w8", 1));
  CHECK(GangScheduler::place_group(group, nodes).empty());  // 9 GPUs do not fit: nothing placed
  nodes[0].used_gpus = {0, 1};
  std::vector<Json> small = {pod("a", 2), pod("b", 4)};
  auto p2 = GangScheduler::place_group(small, nodes);
  CHECK_EQ(p2.size(), (size_t)2);
  for (auto& kv : p2)
    for (int g : kv.second.second) CHECK(g >= 2);
}

TEST(topology_best_fit_numa_placement) {
  NodeInfo n;
  n.name = "n0";
  n.gpus = 8;
  n.gpu_numa = parse_int_list("0,0,0,0,1,1,1,1");
  auto v = pick_gpus(n, 4);
  CHECK(v == std::vector<int>({0, 1, 2, 3}));
  n.used_gpus = {0};
  CHECK(pick_gpus(n, 4) == std::vector<int>({4, 5, 6, 7}));  // domain 0 has only 3 free
  n.used_gpus = {0, 1, 4};
  CHECK(pick_gpus(n, 2) == std::vector<int>({2, 3}));        // best fit: the fuller domain
  n.used_gpus = {};
  auto six = pick_gpus(n, 6);
  CHECK_EQ(six.size(), (size_t)6);
  int d0 = 0;
  for (int g : six) d0 += g < 4;
  CHECK(d0 == 4 || d0 == 2);  // one whole domain + 2 of the other
  // a gang of four 1-GPU pods packs onto one socket
  auto pod = [](const std::string& nm) {
    Json p = J(R"({"metadata":{"name":""},"spec":{"containers":[{"name":"t","resources":{"limits":{"amd.com/gpu":1}}}]}})");
    p["metadata"]["name"] = nm;
    return p;
  };
  std::vector<NodeInfo> nodes = {n};
  nodes[0].used_gpus = {5};
  auto pl = GangScheduler::place_group({pod("a"), pod("b"), pod("c"), pod("d")}, nodes);
  std::set<int> doms;
  for (auto& kv : pl) doms.insert(n.gpu_numa[kv.second.second[0]]);
  CHECK_EQ(doms.size(), (size_t)1);
  CHECK_EQ(*doms.begin(), 0);  // domain 1 has a used GPU -> the whole gang fits only on domain 0
  NodeInfo flat;  // no topology published: one domain, lowest ids
  flat.gpus = 4;
  flat.used_gpus = {1};
  CHECK(pick_gpus(flat, 2) == std::vector<int>({0, 2}));
}

TEST(numa_cpu_pinning_sets) {
  CHECK(parse_cpulist("0-3,8,10-11") == std::vector<int>({0, 1, 2, 3, 8, 10, 11}));
  CHECK(parse_cpulist("").empty());
  Topology t;
  t.gpu_numa = {0, 0, 1, 1};
  t.numa_cpus = {parse_cpulist("0-1,4-5"), parse_cpulist("2-3,6-7")};
  CHECK(cpus_for_gpus(t, {1}) == std::vector<int>({0, 1, 4, 5}));
  CHECK(cpus_for_gpus(t, {0, 3}) == std::vector<int>({0, 1, 2, 3, 4, 5, 6, 7}));
  CHECK(cpus_for_gpus(t, {}).empty());
  CHECK(cpus_for_gpus(Topology{}, {0}).empty());  // unknown topology: no pinning
}

// ----------------------------------------------------------------------------- trainer (reconcile)
namespace {
struct Harness {
  std::shared_ptr<Store> store = new_store();
  std::shared_ptr<FakeClient> c = std::make_shared<FakeClient>(store);
  std::shared_ptr<EventRecorder> rec = std::make_shared<EventRecorder>(c);
  TrainerOptions opts;
  Trainer tr{c, rec, opts};
  Json job(const std::string& name) {
    Json out;
    store->get("tfjobs", "default", name, &out);
    return out;
  }
  std::vector<Json> list(const std::string& plural) {
    ListResult lr;
    c->list(plural, "default", "", "", &lr);
    return lr.items;
  }
  ReconcileResult sync(const std::string& name) { return tr.reconcile(job(name), list("pods"), list("services")); }
  void set_pod_exit(const std::string& pod, int code, const std::string& reason = "") {
    Json p;
    store->get("pods", "default", pod, &p);
    Json cs = Json::object();
    cs["name"] = "tensorflow";
    cs["restartCount"] = 0;
    if (code < 0) {
      cs["state"]["running"]["startedAt"] = "2026-01-01T00:00:00Z";
      p["status"]["phase"] = "Running";
    } else {
      cs["state"]["terminated"]["exitCode"] = code;
      cs["state"]["terminated"]["reason"] = reason.empty() ? (code == 0 ? "Completed" : "Error") : reason;
      p["status"]["phase"] = code == 0 ? "Succeeded" : "Failed";
    }
    p["status"]["containerStatuses"] = Json::array();
    p["status"]["containerStatuses"].push_back(cs);
    Json out;
    CHECK(store->update("pods", "default", pod, p, true, &out).ok());
  }
  std::string cond(const std::string& name) {
    Json j = job(name);
    std::string last;
    for (auto& c2 : j.path("status.conditions").items())
      if (c2.at("status").str() == "True") last = c2.at("type").str();
    return last;
  }
};
}  // namespace

TEST(trainer_creates_pods_services_with_tf_config) {
  Harness h;
  Json out;
  CHECK(h.store->create("tfjobs", "default", v1_job("mnist", 2, 1), &out).ok());
  for (int i = 0; i < 3; ++i) h.sync("mnist");  // setup (finalizer/defaults) then create
  auto pods = h.list("pods");
  auto svcs = h.list("services");
  CHECK_EQ(pods.size(), (size_t)4);
  CHECK_EQ(svcs.size(), (size_t)4);
  bool saw_worker1 = false;
  for (auto& p : pods) {
    std::string tf;
    for (auto& e : p.path("spec.containers")[0].at("env").items())
      if (e.at("name").str() == "TF_CONFIG") tf = e.at("value").str();
    CHECK(!tf.empty());
    Json t = Json::parse(tf);
    if (t.path("task.type").str() == "worker" && t.path("task.index").as_int() == 1) saw_worker1 = true;
    CHECK_EQ(p.path("metadata.ownerReferences")[0].at("kind").str(), std::string("TFJob"));
  }
  CHECK(saw_worker1);
  Json j = h.job("mnist");
  bool fin = false;
  for (auto& f : j.path("metadata.finalizers").items()) fin |= f.str() == api::kFinalizer;
  CHECK(fin);
}

TEST(trainer_success_follows_chief) {
  Harness h;
  Json out;
  h.store->create("tfjobs", "default", v1_job("ok", 1), &out);
  for (int i = 0; i < 3; ++i) h.sync("ok");
  for (auto& p : h.list("pods")) h.set_pod_exit(p.path("metadata.name").str(), -1);
  h.sync("ok");
  CHECK_EQ(h.cond("ok"), std::string("Running"));
  for (auto& p : h.list("pods"))
    if (p.path("metadata.name").str().find("chief") != std::string::npos) h.set_pod_exit(p.path("metadata.name").str(), 0);
  h.sync("ok");
  CHECK_EQ(h.cond("ok"), std::string("Succeeded"));
}

TEST(trainer_retryable_failure_restarts_gang) {
  Harness h;
  Json out;
  h.store->create("tfjobs", "default", v1_job("flaky", 2), &out);
  for (int i = 0; i < 3; ++i) h.sync("flaky");
  for (auto& p : h.list("pods")) h.set_pod_exit(p.path("metadata.name").str(), -1);
  h.sync("flaky");
  h.set_pod_exit("flaky-worker-1", 137);
  for (int i = 0; i < 3; ++i) h.sync("flaky");
  Json j = h.job("flaky");
  bool restarting = false;
  for (auto& c2 : j.path("status.conditions").items()) restarting |= c2.at("type").str() == "Restarting";
  CHECK(restarting);
  CHECK(h.cond("flaky") != "Failed");
  // the whole gang comes back with a bumped restart generation
  auto pods = h.list("pods");
  CHECK_EQ(pods.size(), (size_t)3);
  for (auto& p : pods) {
    std::string gen;
    for (auto& e : p.path("spec.containers")[0].at("env").items())
      if (e.at("name").str() == "TFK_RESTART_GENERATION") gen = e.at("value").str();
    CHECK_EQ(gen, std::string("1"));
  }
}

TEST(trainer_permanent_failure_fails_job) {
  Harness h;
  Json out;
  h.store->create("tfjobs", "default", v1_job("bad", 1), &out);
  for (int i = 0; i < 3; ++i) h.sync("bad");
  h.set_pod_exit("bad-worker-0", 1);
  for (int i = 0; i < 2; ++i) h.sync("bad");
  CHECK_EQ(h.cond("bad"), std::string("Failed"));
}

TEST(trainer_oom_is_permanent) {
  Harness h;
  Json out;
  h.store->create("tfjobs", "default", v1_job("oom", 1), &out);
  for (int i = 0; i < 3; ++i) h.sync("oom");
  h.set_pod_exit("oom-chief-0", 137, "OOMKilled");
  for (int i = 0; i < 2; ++i) h.sync("oom");
  CHECK_EQ(h.cond("oom"), std::string("Failed"));
}

TEST(trainer_cleanup_and_finalizer_on_delete) {
  Harness h;
  Json out;
  h.store->create("tfjobs", "default", v1_job("del", 1), &out);
  for (int i = 0; i < 3; ++i) h.sync("del");
  CHECK(!h.list("pods").empty());
  CHECK(h.store->remove("tfjobs", "default", "del", "Background", &out).ok());
  for (int i = 0; i < 3; ++i) {
    Json j;
    if (h.store->get("tfjobs", "default", "del", &j).code == 404) break;
    h.tr.reconcile(j, h.list("pods"), h.list("services"));
  }
  CHECK_EQ(h.store->get("tfjobs", "default", "del", &out).code, 404);
  CHECK(h.list("pods").empty());
  CHECK(h.list("services").empty());
}

// ----------------------------------------------------------------------------- TF bundle checkpoint
TEST(tf_bundle_roundtrip) {
  char tmpl[] = "/tmp/tfk-ut-XXXXXX";
  std::string dir = mkdtemp(tmpl);
  std::vector<float> w = {1.f, -2.f, 3.5f, 0.25f, 7.f, 8.f};
  int64_t step = 42;
  std::vector<ckpt::TensorRef> ts = {{"dense/kernel", ckpt::DT_FLOAT, {2, 3}, w.data(), w.size() * 4},
                                     {"global_step", ckpt::DT_INT64, {}, &step, 8}};
  std::string err;
  CHECK(ckpt::write_bundle(dir + "/model.ckpt-42", ts, &err));
  CHECK(ckpt::write_checkpoint_state(dir, "model.ckpt-42", {"model.ckpt-42"}, &err));
  ckpt::BundleReader r;
  CHECK(r.open(dir + "/model.ckpt-42", &err));
  CHECK(r.has("dense/kernel") && r.has("global_step"));
  CHECK_EQ(r.entries().at("dense/kernel").shape.size(), (size_t)2);
  std::string bytes;
  CHECK(r.read("dense/kernel", &bytes, &err));
  CHECK_EQ(bytes.size(), (size_t)24);
  CHECK(std::memcmp(bytes.data(), w.data(), 24) == 0);
  std::string latest;
  std::vector<std::string> all;
  CHECK(ckpt::read_checkpoint_state(dir, &latest, &all));
  CHECK_EQ(latest, std::string("model.ckpt-42"));
  // corrupting the data file is detected by the crc
  std::string data = dir + "/model.ckpt-42.data-00000-of-00001";
  FILE* f = fopen(data.c_str(), "r+b");
  CHECK(f != nullptr);
  fseek(f, 4, SEEK_SET);
  fputc(0x7f, f);
  fclose(f);
  ckpt::BundleReader r2;
  CHECK(r2.open(dir + "/model.ckpt-42", &err));
  CHECK(!r2.read("dense/kernel", &bytes, &err));
  std::string cmd = "rm -rf " + dir;
  CHECK(system(cmd.c_str()) == 0);
}

TEST(kubelet_quantities_and_probe_specs) {
  CHECK_EQ(parse_bytes("128Mi"), 128LL << 20);
  CHECK_EQ(parse_bytes("2Gi"), 2LL << 30);
  CHECK_EQ(parse_bytes("1G"), 1000000000LL);
  CHECK_EQ(parse_bytes("1500k"), 1500000LL);
  CHECK_EQ(parse_bytes("4096"), 4096LL);
  CHECK_EQ(parse_bytes("12Qi"), -1LL);
  CHECK_EQ(parse_bytes(""), -1LL);
  Json ctr = Json::parse(R"({"name":"tensorflow","ports":[{"name":"http","containerPort":8080}]})");
  ProbeSpec h = ProbeSpec::parse(Json::parse(R"({"httpGet":{"port":"http","path":"healthz"},"periodSeconds":2})"), ctr);
  CHECK_EQ(h.kind, std::string("http"));
  CHECK_EQ(h.port, 8080);
  CHECK_EQ(h.path, std::string("/healthz"));
  CHECK_EQ(h.period_ms, (int64_t)2000);
  CHECK_EQ(h.timeout_ms, (int64_t)1000);  // Kubernetes defaults
  CHECK_EQ(h.failure_threshold, 3);
  CHECK(!ProbeSpec::parse(Json(), ctr).enabled());
}

TEST(kubelet_probe_handlers) {
  auto wait = [](std::shared_ptr<ProbeSlot> s) {
    for (int i = 0; i < 400 && s->state.load() == 0; ++i) usleep(10000);
    return s->state.load();
  };
  std::vector<std::string> env = {"PATH=/usr/bin:/bin"};
  ProbeSpec ok;
  ok.kind = "exec";
  ok.command = {"true"};
  CHECK_EQ(wait(launch_probe(ok, env)), 1);
  ProbeSpec bad = ok;
  bad.command = {"sh", "-c", "exit 3"};
  auto sb = launch_probe(bad, env);
  CHECK_EQ(wait(sb), 2);
  CHECK(sb->message.find("exited with 3") != std::string::npos);
  ProbeSpec slow = ok;
  slow.command = {"sleep", "5"};
  slow.timeout_ms = 100;
  auto ss = launch_probe(slow, env);
  CHECK_EQ(wait(ss), 2);
  CHECK(ss->message.find("timed out") != std::string::npos);
  // tcp: a listening socket passes, a closed port fails
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  CHECK(bind(fd, (sockaddr*)&a, sizeof a) == 0 && listen(fd, 4) == 0);
  socklen_t l = sizeof a;
  getsockname(fd, (sockaddr*)&a, &l);
  ProbeSpec t;
  t.kind = "tcp";
  t.port = ntohs(a.sin_port);
  CHECK_EQ(wait(launch_probe(t, env)), 1);
  close(fd);
  CHECK_EQ(wait(launch_probe(t, env)), 2);
}

int main(int argc, char** argv) { return tfk_test::run_all(argc, argv); }
