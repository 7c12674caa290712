{{/* Parity: ramalama-models/helm-chart/templates/_helpers.tpl (name/fullname/labels) */}}
{{- define "gguf.name" -}}
{{- default .Chart.Name .Values.nameOverride | trunc 63 | trimSuffix "-" }}
{{- end }}

{{- define "gguf.fullname" -}}
{{- if .Values.fullnameOverride }}
{{- .Values.fullnameOverride | trunc 63 | trimSuffix "-" }}
{{- else }}
{{- $name := default .Chart.Name .Values.nameOverride }}
{{- if contains $name .Release.Name }}
{{- .Release.Name | trunc 63 | trimSuffix "-" }}
{{- else }}
{{- printf "%s-%s" .Release.Name $name | trunc 63 | trimSuffix "-" }}
{{- end }}
{{- end }}
{{- end }}

{{- define "gguf.chart" -}}
{{- printf "%s-%s" .Chart.Name .Chart.Version | replace "+" "_" | trunc 63 | trimSuffix "-" }}
{{- end }}

{{- define "gguf.labels" -}}
helm.sh/chart: {{ include "gguf.chart" . }}
{{ include "gguf.selectorLabels" . }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
{{- end }}

{{- define "gguf.selectorLabels" -}}
app.kubernetes.io/name: {{ include "gguf.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end }}

{{/* per-model resource name: <fullname>-<modelName> (unique per release) */}}
{{- define "gguf.modelName" -}}
{{- printf "%s-%s" (include "gguf.fullname" .root) .model.modelName | trunc 63 | trimSuffix "-" }}
{{- end }}

{{- define "gguf.webui.fullname" -}}
{{- printf "%s-webui" (include "gguf.fullname" .) | trunc 63 | trimSuffix "-" }}
{{- end }}

{{- define "gguf.webui.selectorLabels" -}}
app.kubernetes.io/name: {{ include "gguf.name" . }}-webui
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end }}
