{{/* Common names and labels for amd-gpu-stack. */}}
{{- define "amdgpu.fullname" -}}
{{- .Release.Name | trunc 50 | trimSuffix "-" -}}
{{- end -}}

{{- define "amdgpu.labels" -}}
app.kubernetes.io/part-of: amd-gpu-stack
app.kubernetes.io/managed-by: {{ .Release.Service }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
helm.sh/chart: {{ printf "%s-%s" .Chart.Name .Chart.Version }}
{{- end -}}

{{- define "amdgpu.image" -}}
{{ .Values.image.repository }}:{{ .Values.image.tag }}
{{- end -}}

{{- define "amdgpu.podCommon" -}}
{{- with .Values.imagePullSecrets }}
imagePullSecrets:
{{ toYaml . }}
{{- end }}
{{- with .Values.nodeSelector }}
nodeSelector:
{{ toYaml . | indent 2 }}
{{- end }}
{{- with .Values.tolerations }}
tolerations:
{{ toYaml . }}
{{- end }}
{{- end -}}

{{/* RCCL environment (rccl.profile + rccl.env) as container env items at the
     validator's indentation; must match mxk8s/parallel/rccl_env.py PROFILES
     (tests/test_chart.py checks it). */}}
{{- define "amdgpu.rcclEnv" -}}
{{- $extra := .Values.rccl.env | default (dict) -}}
{{- if eq .Values.rccl.profile "xgmi-node" }}
{{- range $k, $v := dict "NCCL_IB_DISABLE" "1" "HSA_NO_SCRATCH_RECLAIM" "1" "TORCH_NCCL_HIGH_PRIORITY" "1" }}
{{- if not (hasKey $extra $k) }}
            - name: {{ $k }}
              value: {{ $v | quote }}
{{- end }}
{{- end }}
{{- end }}
{{- range $k, $v := $extra }}
            - name: {{ $k }}
              value: {{ $v | quote }}
{{- end }}
{{- end -}}
