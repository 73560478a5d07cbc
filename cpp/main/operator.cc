// tfk-operator: the TFJob operator binary (cmd/tf_operator/main.go equivalent, images/tf.PNG:L6):
// NewServerOption -> AddFlags -> parse + init logging -> Run server (images/tf2.png).
#include <cstdio>

#include "../operator/options.h"

int main(int argc, char** argv) {
  using namespace tfk;
  ServerOption s = ServerOption::New();
  FlagSet fs("tfk-operator");
  s.AddFlags(fs);
  std::string err;
  if (!fs.parse(argc, argv, &err)) { fprintf(stderr, "%s\n%s", err.c_str(), fs.usage().c_str()); return 2; }
  if (fs.help_requested()) { printf("%s", fs.usage().c_str()); return 0; }
  if (s.print_version) { printf("tfk-operator v0.1.0 (TFJob kubeflow.org/v1, v1alpha1)\n"); return 0; }
  InitLogging("tf-operator", s.json_log_format, s.log_level);
  StopToken stop;
  HandleSignals(stop);
  return RunServer(s, stop);
}
