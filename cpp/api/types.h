// TFJob API (reference: pkg/apis/tensorflow/v1alpha1/{types,defaults,register}.go, images/tf3.PNG:L7-L14;
// CRD manifest k8s-operator.md:8-34). One internal hub model serves both wire versions:
//   tensorflow.org|kubeflow.org/v1alpha1 : spec.replicaSpecs[] {replicas, tfPort, tfReplicaType, template},
//                                          status {phase, state, reason, replicaStatuses[]}
//   kubeflow.org/v1                      : spec.tfReplicaSpecs{Chief|Master|PS|Worker|Evaluator}, runPolicy,
//                                          status {conditions[], replicaStatuses{}}
#pragma once
#include <map>
#include <string>
#include <vector>

#include "../common/json.h"

namespace tfk {
namespace api {

constexpr const char* kGroupV1 = "kubeflow.org";
constexpr const char* kGroupV1alpha1Legacy = "tensorflow.org";
constexpr const char* kKind = "TFJob";
constexpr const char* kPlural = "tfjobs";
constexpr const char* kSingular = "tfjob";
constexpr const char* kShortName = "tfj";
constexpr const char* kContainerName = "tensorflow";
constexpr const char* kPortName = "tfjob-port";
// TFJob/pod annotation (any non-empty value): the gang scheduler records the union of the gang's
// GPU ids on a node (tfk.io/gang-gpu-ids) and the kubelet exposes all of them to every member pod
// with TFK_LOCAL_DEVICE = the pod's own index in that list (RCCL then finds its peers for P2P/IPC).
constexpr const char* kGangVisibleGpus = "scheduling.tfk.io/gang-visible-gpus";
constexpr const char* kGangGpuIds = "tfk.io/gang-gpu-ids";
constexpr int kDefaultPort = 2222;
constexpr const char* kFinalizer = "tfjob.kubeflow.org/cleanup";
constexpr const char* kGPUResource = "amd.com/gpu";
// v1alpha1-only spec fields carried as annotations by the v1 storage shape
constexpr const char* kAnnRuntimeId = "tensorflow.org/v1alpha1-runtime-id";
constexpr const char* kAnnTfImage = "tensorflow.org/v1alpha1-tf-image";
constexpr const char* kAnnChief = "tensorflow.org/v1alpha1-termination-chief";

// Canonical (upper-case) replica types. v1alpha1 uses them verbatim; v1 uses Title case.
enum class RType { Master, Chief, PS, Worker, Evaluator, Unknown };
RType rtype_from(const std::string& s);
std::string rtype_upper(RType t);  // MASTER
std::string rtype_title(RType t);  // Master (v1 map key)
std::string rtype_lower(RType t);  // master (TF_CONFIG cluster key / DNS)

struct ReplicaSpec {
  RType type = RType::Master;
  int replicas = -1;          // -1 = unset (defaulted to 1)
  int tf_port = -1;           // -1 = unset (defaulted to 2222)
  std::string restart_policy; // v1: Always|OnFailure|Never|ExitCode ("" = default)
  bool is_default_ps = false; // v1alpha1
  Json template_;             // PodTemplateSpec
};

struct SchedulingPolicy {
  int min_available = -1;
  std::string queue, priority_class;
};

struct RunPolicy {
  std::string clean_pod_policy;  // All|Running|None ("" = default)
  long long ttl_seconds_after_finished = -1;
  long long active_deadline_seconds = -1;
  int backoff_limit = -1;
  SchedulingPolicy scheduling;
};

struct JobCondition {
  std::string type, status, reason, message, last_update, last_transition;
};

struct ReplicaStatus {
  int active = 0, succeeded = 0, failed = 0;
  std::string state;                 // v1alpha1 ReplicaState: Unknown|Running|Succeeded|Failed
  std::map<std::string, int> states; // v1alpha1 replicas_states
};

struct TFJobStatus {
  std::string phase;  // v1alpha1: ""|Creating|Running|CleanUp|Failed|Done
  std::string state;  // v1alpha1: Unknown|Running|Succeeded|Failed
  std::string reason;
  std::vector<JobCondition> conditions;
  std::map<RType, ReplicaStatus> replica_statuses;
  std::string start_time, completion_time, last_reconcile_time;
  int restart_count = 0;  // gang restarts after retryable failures (counted against backoffLimit)
  int resize_count = 0;   // coordinated restarts after a replica-count change (not counted)
};

struct TFJob {
  std::string api_version = "kubeflow.org/v1";
  Json metadata;
  // spec
  std::string runtime_id, tf_image, scheduler_name;
  std::string chief_name;   // termination policy chief replica type (upper), "" = default
  int chief_index = -1;
  bool has_termination_policy = false;
  std::vector<ReplicaSpec> replicas;  // ordered as given
  RunPolicy run_policy;
  std::string success_policy;  // ""|AllWorkers
  TFJobStatus status;

  bool is_v1alpha1() const;
  std::string name() const { return metadata.at("name").str(); }
  std::string ns() const { return metadata.at("namespace").str("default"); }
  std::string uid() const { return metadata.at("uid").str(); }
  const ReplicaSpec* replica(RType t) const;
  ReplicaSpec* replica(RType t);
};

// Codec
TFJob from_json(const Json& j);                 // throws std::runtime_error on malformed input
Json to_json(const TFJob& job);                 // in job.api_version's wire shape
Json convert(const Json& obj, const std::string& target_api_version);  // v1alpha1 <-> v1

// Defaulting (defaults.go SetDefaults_TFJob) and validation (validation.go ValidateTFJobSpec).
void set_defaults(TFJob& job);
std::vector<std::string> validate(const TFJob& job);  // empty == valid

// Helpers (helper/helpers.go)
std::string crd_name();  // "<plural>.<group>"
Json crd_manifest();     // apiextensions.k8s.io/v1beta1 CustomResourceDefinition
Json as_owner(const TFJob& job);  // OwnerReference{controller:true, blockOwnerDeletion:true}

struct AcceleratorConfig {
  std::vector<std::pair<std::string, std::pair<std::string, std::string>>> volumes;  // name -> (hostPath, mountPath)
  std::vector<std::pair<std::string, std::string>> env;
};
struct ControllerConfig {
  std::map<std::string, AcceleratorConfig> accelerators;  // resource name -> config
  std::string grpc_server_file_path;                      // default-PS script (v1alpha1 isDefaultPS)
  static ControllerConfig defaults();                     // amd.com/gpu -> /dev/kfd, /dev/dri
  static ControllerConfig from_json(const Json& j);
};
// Inject hostPath volumes/mounts + env for every accelerator resource requested by the
// "tensorflow" container of each replica template (ConfigureAcceleratorsForTFJobSpec).
void configure_accelerators(TFJob& job, const ControllerConfig& cfg);

// Names / TF_CONFIG
std::string gen_name(const TFJob& job, RType t, int index);  // DNS-1123, job name truncated to 40
std::string gen_general_name(const std::string& job_name, const std::string& rtype_lower, int index);
Json cluster_spec(const TFJob& job, const std::string& cluster_domain, const std::map<std::string, int>* ports);
std::string tf_config(const TFJob& job, RType t, int index, const std::string& cluster_domain,
                      const std::map<std::string, int>* ports = nullptr);

// Status helpers
void set_condition(TFJobStatus& st, const std::string& type, const std::string& reason, const std::string& msg,
                   const std::string& now);
bool has_condition(const TFJobStatus& st, const std::string& type);
bool is_finished(const TFJobStatus& st);
// Exit-code classification (training.go isRetryableTerminationState): 0 success, 1-127 permanent,
// >=128 (signals: 137 SIGKILL, 143 SIGTERM) retryable, OOMKilled permanent.
bool is_retryable_exit(int exit_code, const std::string& reason);

}  // namespace api
}  // namespace tfk
