"""``ray.serve.gradio_integrations`` (reference: python/ray/serve/gradio_integrations.py):
serve a Gradio app as a deployment. Each replica calls ``builder()`` for the Gradio
Blocks/Interface and serves its ASGI app (the replica routes HTTP requests to an ASGI app
its constructor sets, serve/_replica.py). ``gradio`` is not installed in this image:
constructing the ingress then raises ImportError naming it."""

from __future__ import annotations

from ray_amd import serve


class GradioIngress:
    def __init__(self, builder):
        try:
            import gradio as gr
        except ImportError as e:
            raise ImportError("GradioIngress needs the 'gradio' package, which is not "
                              "installed") from e
        from fastapi import FastAPI

        app = FastAPI()
        self._serve_asgi_instance_app = gr.mount_gradio_app(app, builder(), path="/")


GradioServer = serve.deployment(GradioIngress, name="GradioServer")
