// YAML subset -> Json, enough for kubeconfig files and Kubernetes manifests written by kubectl /
// humans: block mappings and sequences (including "key:\n- item" at the key's indent), plain /
// single- / double-quoted scalars with YAML 1.2 core-schema typing (true/false/null/~/ints/floats),
// flow sequences and mappings of scalars ([a, b], {k: v}), literal (|) and folded (>) block
// scalars, comments and a leading "---". Anchors, aliases, tags and multi-document streams are
// rejected with an error rather than mis-parsed.
#pragma once
#include <string>
#include <vector>

#include "json.h"

namespace tfk {

Json yaml_parse(const std::string& text);  // throws std::runtime_error("yaml: line N: ...")
// Split a multi-document stream on "---" lines and parse each non-empty document.
std::vector<Json> yaml_parse_all(const std::string& text);

}  // namespace tfk
