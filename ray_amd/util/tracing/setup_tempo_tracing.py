"""``ray.util.tracing.setup_tempo_tracing`` (reference path): export to a Grafana Tempo
OTLP endpoint. It needs the OpenTelemetry SDK and exporter, which are not installed; the
built-in JSON-lines exporter (``setup_local_tmp_tracing``) is the available one."""


def setup_tracing() -> None:
    try:
        import opentelemetry  # noqa: F401
    except ImportError as e:
        raise ImportError("setup_tempo_tracing needs 'opentelemetry-sdk' and the OTLP "
                          "exporter, which are not installed") from e
    raise NotImplementedError("OTLP export is not wired; use setup_local_tmp_tracing")
