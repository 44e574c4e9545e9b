"""Flask app (web/__init__.py of the reference): GET /?cube_name=&num_recs=&root=.  Serving is out of
the hot-path scope; the app is kept only as the caller of get_ml_recommend."""
