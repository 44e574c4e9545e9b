"""The reference's Flask endpoint (web/__init__.py: GET /?cube_name=&num_recs=&root=) over this
package's get_ml_recommend.  HTTP serving is outside the hot-path scope; the app is
the caller the boundary keeps: the same query parameters, defaults (num_recs 30000, root
cubecobra.com), error strings and jsonify'd result.  Flask's threads share the one resident model
(web/ml_recommend_web.py -> api.get_model); every request's forward + top-N runs on the GPU."""
import logging

from flask import Flask, jsonify, request

from .ml_recommend_web import get_ml_recommend

app = Flask(__name__)
DEFAULT_NUM_RECS = 30000                      # rank every card (>= |V|)
DEFAULT_ROOT = 'https://www.cubecobra.com'

if __name__ != '__main__':                    # under gunicorn: its error log carries ours
    app.logger.handlers.extend(logging.getLogger('gunicorn.error').handlers)
    app.logger.setLevel(logging.DEBUG)


@app.route('/')
def api():
    cube_name = request.args.get('cube_name')
    num_recs = request.args.get('num_recs', DEFAULT_NUM_RECS)
    root = request.args.get('root', DEFAULT_ROOT)
    if not (cube_name and num_recs):
        msg = 'Need cube_name and num_recs as parameters!'
        app.logger.error(msg)
        return msg
    try:
        num_recs = int(num_recs)
    except ValueError:
        msg = 'num_recs needs to be an integer!'
        app.logger.error(msg)
        return msg
    return jsonify(get_ml_recommend(cube_name, num_recs, root))


if __name__ == '__main__':
    app.run(host='0.0.0.0', port=8000, threaded=True)
