// Kubernetes manifests of a service graph (isotope convert/pkg/kubernetes);
// see k8s.cpp.
#pragma once
#include <string>

#include "../../include/isim.h"
#include "graph.h"

namespace isim {

// yaml.Marshal(graph) through sigs.k8s.io/yaml (JSONToYAML of json.Marshal):
// the ConfigMap payload of kubernetes.go:159-175.  Empty on failure.
std::string graph_yaml(const ServiceGraph &g);

// ServiceGraphToKubernetesManifests (kubernetes.go:56-137).
int k8s_manifests(const ServiceGraph &g, const isim_k8s_params &p, std::string &out, std::string &err);

}  // namespace isim
