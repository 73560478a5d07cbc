// tfk-scheduler: gang scheduler for TFJob pods (amd.com/gpu, all-or-nothing).
#include <cstdio>

#include "../operator/options.h"
#include "../scheduler/scheduler.h"

int main(int argc, char** argv) {
  using namespace tfk;
  std::string apiserver = "http://127.0.0.1:8080", name = "tfk-gang", level = "info";
  bool json = false, default_too = true;
  FlagSet fs("tfk-scheduler");
  fs.add_string("apiserver", &apiserver, "apiserver URL");
  fs.add_string("scheduler-name", &name, "schedulerName to serve");
  fs.add_bool("schedule-default", &default_too, "also schedule pods without a scheduler name");
  fs.add_bool("json-log-format", &json, "JSON logs");
  fs.add_string("log-level", &level, "log level");
  std::string err;
  if (!fs.parse(argc, argv, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 2; }
  InitLogging("tfk-scheduler", json, level);
  StopToken stop;
  HandleSignals(stop);
  RestConfig rc;
  rc.host = apiserver;
  rc.qps = 100;
  rc.burst = 200;
  SchedulerOptions so;
  so.name = name;
  so.schedule_default = default_too;
  GangScheduler s(new_for_config(rc), so);
  s.run(stop);
  return 0;
}
