// Field types of the objects validatePodSecurity decodes (pkg/engine/validation.go:481-532 getSpec: json.Unmarshal of
// the whole resource into corev1.Pod, appsv1.Deployment -- for every workload kind -- or batchv1.CronJob), restated
// from the published Go types of k8s.io/api v0.26.1 (core/v1, apps/v1, batch/v1) and k8s.io/apimachinery v0.26.1
// (meta/v1 ObjectMeta / LabelSelector / Time, api/resource Quantity, util/intstr IntOrString). Neither module is
// vendored under /root/reference: this table is parity-unpinned data, read by the flattener's typed decode
// (batch.cpp, RF_PSS_DEC_ERR) and, through its own decoder, by the oracle (oracle/otyped.cpp).
//
// One struct per line: `Name{field:type ...}` or `Name:Base{...}` (Base's fields promoted: Go embedded structs with
// `json:",inline"`). Types:
//   s string   b bool   i32 / i64 integer (json number literal parsed by strconv.ParseInt, range checked)
//   q  resource.Quantity (UnmarshalJSON: a string or number literal that ParseQuantity accepts)
//   ios intstr.IntOrString (a string, or an int32 literal)   t metav1.Time (a string time.Parse(RFC3339) accepts)
//   any  metav1.FieldsV1 (raw JSON: anything)   [T] slice of T   {T} map[string]T   Name a struct
// Pointers and values decode alike (null leaves the zero value); unknown fields are ignored; a key matches its field
// exactly, else ASCII case-insensitively (encoding/json's fold match).
#pragma once

namespace k8st {

inline const char* kSchema = R"(
Pod{kind:s apiVersion:s metadata:ObjectMeta spec:PodSpec status:PodStatus}
Deployment{kind:s apiVersion:s metadata:ObjectMeta spec:DeploymentSpec status:DeploymentStatus}
CronJob{kind:s apiVersion:s metadata:ObjectMeta spec:CronJobSpec status:CronJobStatus}
ObjectMeta{name:s generateName:s namespace:s selfLink:s uid:s resourceVersion:s generation:i64 creationTimestamp:t deletionTimestamp:t deletionGracePeriodSeconds:i64 labels:{s} annotations:{s} ownerReferences:[OwnerReference] finalizers:[s] managedFields:[ManagedFieldsEntry]}
OwnerReference{apiVersion:s kind:s name:s uid:s controller:b blockOwnerDeletion:b}
ManagedFieldsEntry{manager:s operation:s apiVersion:s time:t fieldsType:s fieldsV1:any subresource:s}
LabelSelector{matchLabels:{s} matchExpressions:[LabelSelectorRequirement]}
LabelSelectorRequirement{key:s operator:s values:[s]}
PodSpec{volumes:[Volume] initContainers:[Container] containers:[Container] ephemeralContainers:[EphemeralContainer] restartPolicy:s terminationGracePeriodSeconds:i64 activeDeadlineSeconds:i64 dnsPolicy:s nodeSelector:{s} serviceAccountName:s serviceAccount:s automountServiceAccountToken:b nodeName:s hostNetwork:b hostPID:b hostIPC:b shareProcessNamespace:b securityContext:PodSecurityContext imagePullSecrets:[LocalObjectReference] hostname:s subdomain:s affinity:Affinity schedulerName:s tolerations:[Toleration] hostAliases:[HostAlias] priorityClassName:s priority:i32 dnsConfig:PodDNSConfig readinessGates:[PodReadinessGate] runtimeClassName:s enableServiceLinks:b preemptionPolicy:s overhead:{q} topologySpreadConstraints:[TopologySpreadConstraint] setHostnameAsFQDN:b os:PodOS hostUsers:b schedulingGates:[PodSchedulingGate] resourceClaims:[PodResourceClaim]}
Container{name:s image:s command:[s] args:[s] workingDir:s ports:[ContainerPort] envFrom:[EnvFromSource] env:[EnvVar] resources:ResourceRequirements volumeMounts:[VolumeMount] volumeDevices:[VolumeDevice] livenessProbe:Probe readinessProbe:Probe startupProbe:Probe lifecycle:Lifecycle terminationMessagePath:s terminationMessagePolicy:s imagePullPolicy:s securityContext:SecurityContext stdin:b stdinOnce:b tty:b}
EphemeralContainer:Container{targetContainerName:s}
ContainerPort{name:s hostPort:i32 containerPort:i32 protocol:s hostIP:s}
EnvFromSource{prefix:s configMapRef:ConfigMapEnvSource secretRef:SecretEnvSource}
LocalObjectReference{name:s}
ConfigMapEnvSource:LocalObjectReference{optional:b}
SecretEnvSource:LocalObjectReference{optional:b}
EnvVar{name:s value:s valueFrom:EnvVarSource}
EnvVarSource{fieldRef:ObjectFieldSelector resourceFieldRef:ResourceFieldSelector configMapKeyRef:ConfigMapKeySelector secretKeyRef:SecretKeySelector}
ObjectFieldSelector{apiVersion:s fieldPath:s}
ResourceFieldSelector{containerName:s resource:s divisor:q}
ConfigMapKeySelector:LocalObjectReference{key:s optional:b}
SecretKeySelector:LocalObjectReference{key:s optional:b}
ResourceRequirements{limits:{q} requests:{q} claims:[ResourceClaim]}
ResourceClaim{name:s}
VolumeMount{name:s readOnly:b mountPath:s subPath:s mountPropagation:s subPathExpr:s}
VolumeDevice{name:s devicePath:s}
ProbeHandler{exec:ExecAction httpGet:HTTPGetAction tcpSocket:TCPSocketAction grpc:GRPCAction}
Probe:ProbeHandler{initialDelaySeconds:i32 timeoutSeconds:i32 periodSeconds:i32 successThreshold:i32 failureThreshold:i32 terminationGracePeriodSeconds:i64}
ExecAction{command:[s]}
HTTPGetAction{path:s port:ios host:s scheme:s httpHeaders:[HTTPHeader]}
HTTPHeader{name:s value:s}
TCPSocketAction{port:ios host:s}
GRPCAction{port:i32 service:s}
Lifecycle{postStart:LifecycleHandler preStop:LifecycleHandler}
LifecycleHandler{exec:ExecAction httpGet:HTTPGetAction tcpSocket:TCPSocketAction}
SecurityContext{capabilities:Capabilities privileged:b seLinuxOptions:SELinuxOptions windowsOptions:WindowsSecurityContextOptions runAsUser:i64 runAsGroup:i64 runAsNonRoot:b readOnlyRootFilesystem:b allowPrivilegeEscalation:b procMount:s seccompProfile:SeccompProfile}
Capabilities{add:[s] drop:[s]}
SELinuxOptions{user:s role:s type:s level:s}
WindowsSecurityContextOptions{gmsaCredentialSpecName:s gmsaCredentialSpec:s runAsUserName:s hostProcess:b}
SeccompProfile{type:s localhostProfile:s}
PodSecurityContext{seLinuxOptions:SELinuxOptions windowsOptions:WindowsSecurityContextOptions runAsUser:i64 runAsGroup:i64 runAsNonRoot:b supplementalGroups:[i64] fsGroup:i64 sysctls:[Sysctl] fsGroupChangePolicy:s seccompProfile:SeccompProfile}
Sysctl{name:s value:s}
Affinity{nodeAffinity:NodeAffinity podAffinity:PodAffinity podAntiAffinity:PodAntiAffinity}
NodeAffinity{requiredDuringSchedulingIgnoredDuringExecution:NodeSelector preferredDuringSchedulingIgnoredDuringExecution:[PreferredSchedulingTerm]}
NodeSelector{nodeSelectorTerms:[NodeSelectorTerm]}
NodeSelectorTerm{matchExpressions:[NodeSelectorRequirement] matchFields:[NodeSelectorRequirement]}
NodeSelectorRequirement{key:s operator:s values:[s]}
PreferredSchedulingTerm{weight:i32 preference:NodeSelectorTerm}
PodAffinity{requiredDuringSchedulingIgnoredDuringExecution:[PodAffinityTerm] preferredDuringSchedulingIgnoredDuringExecution:[WeightedPodAffinityTerm]}
PodAntiAffinity:PodAffinity{}
PodAffinityTerm{labelSelector:LabelSelector namespaces:[s] topologyKey:s namespaceSelector:LabelSelector}
WeightedPodAffinityTerm{weight:i32 podAffinityTerm:PodAffinityTerm}
Toleration{key:s operator:s value:s effect:s tolerationSeconds:i64}
HostAlias{ip:s hostnames:[s]}
PodDNSConfig{nameservers:[s] searches:[s] options:[PodDNSConfigOption]}
PodDNSConfigOption{name:s value:s}
PodReadinessGate{conditionType:s}
TopologySpreadConstraint{maxSkew:i32 topologyKey:s whenUnsatisfiable:s labelSelector:LabelSelector minDomains:i32 nodeAffinityPolicy:s nodeTaintsPolicy:s matchLabelKeys:[s]}
PodOS{name:s}
PodSchedulingGate{name:s}
PodResourceClaim{name:s source:ClaimSource}
ClaimSource{resourceClaimName:s resourceClaimTemplateName:s}
VolumeSource{hostPath:HostPathVolumeSource emptyDir:EmptyDirVolumeSource gcePersistentDisk:GCEPersistentDiskVolumeSource awsElasticBlockStore:AWSElasticBlockStoreVolumeSource gitRepo:GitRepoVolumeSource secret:SecretVolumeSource nfs:NFSVolumeSource iscsi:ISCSIVolumeSource glusterfs:GlusterfsVolumeSource persistentVolumeClaim:PersistentVolumeClaimVolumeSource rbd:RBDVolumeSource flexVolume:FlexVolumeSource cinder:CinderVolumeSource cephfs:CephFSVolumeSource flocker:FlockerVolumeSource downwardAPI:DownwardAPIVolumeSource fc:FCVolumeSource azureFile:AzureFileVolumeSource configMap:ConfigMapVolumeSource vsphereVolume:VsphereVirtualDiskVolumeSource quobyte:QuobyteVolumeSource azureDisk:AzureDiskVolumeSource photonPersistentDisk:PhotonPersistentDiskVolumeSource projected:ProjectedVolumeSource portworxVolume:PortworxVolumeSource scaleIO:ScaleIOVolumeSource storageos:StorageOSVolumeSource csi:CSIVolumeSource ephemeral:EphemeralVolumeSource}
Volume:VolumeSource{name:s}
HostPathVolumeSource{path:s type:s}
EmptyDirVolumeSource{medium:s sizeLimit:q}
GCEPersistentDiskVolumeSource{pdName:s fsType:s partition:i32 readOnly:b}
AWSElasticBlockStoreVolumeSource{volumeID:s fsType:s partition:i32 readOnly:b}
GitRepoVolumeSource{repository:s revision:s directory:s}
SecretVolumeSource{secretName:s items:[KeyToPath] defaultMode:i32 optional:b}
KeyToPath{key:s path:s mode:i32}
NFSVolumeSource{server:s path:s readOnly:b}
ISCSIVolumeSource{targetPortal:s iqn:s lun:i32 iscsiInterface:s fsType:s readOnly:b portals:[s] chapAuthDiscovery:b chapAuthSession:b secretRef:LocalObjectReference initiatorName:s}
GlusterfsVolumeSource{endpoints:s path:s readOnly:b}
PersistentVolumeClaimVolumeSource{claimName:s readOnly:b}
RBDVolumeSource{monitors:[s] image:s fsType:s pool:s user:s keyring:s secretRef:LocalObjectReference readOnly:b}
FlexVolumeSource{driver:s fsType:s secretRef:LocalObjectReference readOnly:b options:{s}}
CinderVolumeSource{volumeID:s fsType:s readOnly:b secretRef:LocalObjectReference}
CephFSVolumeSource{monitors:[s] path:s user:s secretFile:s secretRef:LocalObjectReference readOnly:b}
FlockerVolumeSource{datasetName:s datasetUUID:s}
DownwardAPIVolumeSource{items:[DownwardAPIVolumeFile] defaultMode:i32}
DownwardAPIVolumeFile{path:s fieldRef:ObjectFieldSelector resourceFieldRef:ResourceFieldSelector mode:i32}
FCVolumeSource{targetWWNs:[s] lun:i32 fsType:s readOnly:b wwids:[s]}
AzureFileVolumeSource{secretName:s shareName:s readOnly:b}
ConfigMapVolumeSource:LocalObjectReference{items:[KeyToPath] defaultMode:i32 optional:b}
VsphereVirtualDiskVolumeSource{volumePath:s fsType:s storagePolicyName:s storagePolicyID:s}
QuobyteVolumeSource{registry:s volume:s readOnly:b user:s group:s tenant:s}
AzureDiskVolumeSource{diskName:s diskURI:s cachingMode:s fsType:s readOnly:b kind:s}
PhotonPersistentDiskVolumeSource{pdID:s fsType:s}
ProjectedVolumeSource{sources:[VolumeProjection] defaultMode:i32}
VolumeProjection{secret:SecretProjection downwardAPI:DownwardAPIProjection configMap:ConfigMapProjection serviceAccountToken:ServiceAccountTokenProjection}
SecretProjection:LocalObjectReference{items:[KeyToPath] optional:b}
ConfigMapProjection:LocalObjectReference{items:[KeyToPath] optional:b}
DownwardAPIProjection{items:[DownwardAPIVolumeFile]}
ServiceAccountTokenProjection{audience:s expirationSeconds:i64 path:s}
PortworxVolumeSource{volumeID:s fsType:s readOnly:b}
ScaleIOVolumeSource{gateway:s system:s secretRef:LocalObjectReference sslEnabled:b protectionDomain:s storagePool:s storageMode:s volumeName:s fsType:s readOnly:b}
StorageOSVolumeSource{volumeName:s volumeNamespace:s fsType:s readOnly:b secretRef:LocalObjectReference}
CSIVolumeSource{driver:s readOnly:b fsType:s volumeAttributes:{s} nodePublishSecretRef:LocalObjectReference}
EphemeralVolumeSource{volumeClaimTemplate:PersistentVolumeClaimTemplate}
PersistentVolumeClaimTemplate{metadata:ObjectMeta spec:PersistentVolumeClaimSpec}
PersistentVolumeClaimSpec{accessModes:[s] selector:LabelSelector resources:ResourceRequirements volumeName:s storageClassName:s volumeMode:s dataSource:TypedLocalObjectReference dataSourceRef:TypedObjectReference}
TypedLocalObjectReference{apiGroup:s kind:s name:s}
TypedObjectReference{apiGroup:s kind:s name:s namespace:s}
PodStatus{phase:s conditions:[PodCondition] message:s reason:s nominatedNodeName:s hostIP:s podIP:s podIPs:[PodIP] startTime:t initContainerStatuses:[ContainerStatus] containerStatuses:[ContainerStatus] qosClass:s ephemeralContainerStatuses:[ContainerStatus]}
PodCondition{type:s status:s lastProbeTime:t lastTransitionTime:t reason:s message:s}
PodIP{ip:s}
ContainerStatus{name:s state:ContainerState lastState:ContainerState ready:b restartCount:i32 image:s imageID:s containerID:s started:b}
ContainerState{waiting:ContainerStateWaiting running:ContainerStateRunning terminated:ContainerStateTerminated}
ContainerStateWaiting{reason:s message:s}
ContainerStateRunning{startedAt:t}
ContainerStateTerminated{exitCode:i32 signal:i32 reason:s message:s startedAt:t finishedAt:t containerID:s}
DeploymentSpec{replicas:i32 selector:LabelSelector template:PodTemplateSpec strategy:DeploymentStrategy minReadySeconds:i32 revisionHistoryLimit:i32 paused:b progressDeadlineSeconds:i32}
PodTemplateSpec{metadata:ObjectMeta spec:PodSpec}
DeploymentStrategy{type:s rollingUpdate:RollingUpdateDeployment}
RollingUpdateDeployment{maxUnavailable:ios maxSurge:ios}
DeploymentStatus{observedGeneration:i64 replicas:i32 updatedReplicas:i32 readyReplicas:i32 availableReplicas:i32 unavailableReplicas:i32 conditions:[DeploymentCondition] collisionCount:i32}
DeploymentCondition{type:s status:s lastUpdateTime:t lastTransitionTime:t reason:s message:s}
CronJobSpec{schedule:s timeZone:s startingDeadlineSeconds:i64 concurrencyPolicy:s suspend:b jobTemplate:JobTemplateSpec successfulJobsHistoryLimit:i32 failedJobsHistoryLimit:i32}
JobTemplateSpec{metadata:ObjectMeta spec:JobSpec}
JobSpec{parallelism:i32 completions:i32 activeDeadlineSeconds:i64 podFailurePolicy:PodFailurePolicy backoffLimit:i32 selector:LabelSelector manualSelector:b template:PodTemplateSpec ttlSecondsAfterFinished:i32 completionMode:s suspend:b}
PodFailurePolicy{rules:[PodFailurePolicyRule]}
PodFailurePolicyRule{action:s onExitCodes:PodFailurePolicyOnExitCodesRequirement onPodConditions:[PodFailurePolicyOnPodConditionsPattern]}
PodFailurePolicyOnExitCodesRequirement{containerName:s operator:s values:[i32]}
PodFailurePolicyOnPodConditionsPattern{type:s status:s}
CronJobStatus{active:[ObjectReference] lastScheduleTime:t lastSuccessfulTime:t}
ObjectReference{kind:s namespace:s name:s uid:s apiVersion:s resourceVersion:s fieldPath:s}
)";

}  // namespace k8st
