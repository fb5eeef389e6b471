module isim.local/go

go 1.14

require sigs.k8s.io/yaml v1.2.0
