{{/* Resource-name prefix; unique per release when namePrefix is changed. */}}
{{- define "hf.prefix" -}}{{ .Values.namePrefix | default "hipserve" | trunc 40 | trimSuffix "-" }}{{- end }}
{{- define "hf.gateway" -}}{{ include "hf.prefix" . }}-api-gateway{{- end }}
{{- define "hf.webui" -}}{{ include "hf.prefix" . }}-webui{{- end }}
{{- define "hf.labels" -}}
app.kubernetes.io/managed-by: {{ .Release.Service }}
app.kubernetes.io/part-of: {{ include "hf.prefix" . }}
helm.sh/chart: {{ .Chart.Name }}-{{ .Chart.Version }}
{{- end }}
