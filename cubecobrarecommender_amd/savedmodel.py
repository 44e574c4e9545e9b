"""``saved_model.pb`` of an ``ml_files/<name>/`` export (the checkpoint layout).

Reference: ``autoencoder.save(dest, save_format='tf')`` (src/ml/train.py:112-115) writes a Keras
SavedModel; ``keras.models.load_model`` reads it back (src/scripts/ml_recommend.py:54,
web/ml_recommend_web.py:37).  The file is a ``SavedModel`` proto (tensorflow/core/protobuf/
saved_model.proto) holding one ``MetaGraphDef`` whose ``SavedObjectGraph`` names the same objects,
in the same node order, as the checkpoint's ``_CHECKPOINTABLE_OBJECT_GRAPH``
(checkpoint.object_graph): the loader matches the variables bundle to these nodes.

Written here, without TensorFlow:
  * every node of the checkpoint's object graph, with the same children and slot variables;
  * variable nodes as ``SavedVariable`` {dtype, shape, trainable, synchronization, aggregation,
    name} with the shapes of the tensors in the bundle;
  * the Keras objects as ``SavedUserObject`` {identifier, version, metadata}: the model / Encoder /
    Decoder (``_tf_keras_model``) and Dense layers (``_tf_keras_layer``) with the layer configs of
    src/ml/model.py:20-98 (units, activation, initializers) and the compile() training config of
    train.py:82-88; the optimizer and the metric accumulators (train.py:87);
  * MetaInfoDef tags {"serve"} and a V2 SaverDef naming the variables bundle.
What only TensorFlow can produce — the traced call functions (``SavedConcreteFunction``s and their
GraphDef function library) — is absent, so Keras' loader can revive the Dense layers from their
configs but not call the subclassed model; parity against files TF writes stays unpinned (the
reference's saved_model.pb files are Git-LFS pointers: only their sizes are known, 455,003 B for
cc_rec_1000_regularization).  ``parse_saved_model`` reads the file back (tests/test_checkpoint.py).
"""
import json

from .checkpoint import DT_FLOAT, DT_INT64, OBJECT_GRAPH_KEY, _LAYER_NAMES, _field, _parse, parse_object_graph

SCHEMA_VERSION = 1
PRODUCER = 'ccrec-mi355x/1'
# SavedVariable enums (tensorflow/core/framework/variable.proto)
SYNC_AUTO, SYNC_ON_READ = 0, 3
AGG_NONE, AGG_SUM, AGG_ONLY_FIRST_REPLICA = 0, 1, 3
# the Keras model's sub-model names: Keras names unnamed Model subclasses from the class name,
# the second Decoder instance getting the "_1" suffix (model.py:92-98)
_SUBMODEL = {'encoder': ('Encoder', 'encoder'), 'decoder': ('Decoder', 'decoder'),
             'decoder_for_reg': ('Decoder', 'decoder_1')}


def _dense_meta(name, units, activation, fan_in):
    """Keras' SavedModel metadata of a Dense layer (model.py: Dense(units, activation, name))."""
    cfg = {'name': name, 'trainable': True, 'dtype': 'float32', 'units': int(units), 'activation': activation,
           'use_bias': True, 'kernel_initializer': {'class_name': 'GlorotUniform', 'config': {'seed': None}},
           'bias_initializer': {'class_name': 'Zeros', 'config': {}}, 'kernel_regularizer': None,
           'bias_regularizer': None, 'activity_regularizer': None, 'kernel_constraint': None,
           'bias_constraint': None}
    return {'class_name': 'Dense', 'name': name, 'trainable': True, 'expects_training_arg': False,
            'dtype': 'float32', 'batch_input_shape': None, 'stateful': False, 'must_restore_from_config': False,
            'config': cfg,
            'input_spec': {'class_name': 'InputSpec', 'config': {'dtype': None, 'shape': None, 'ndim': None,
                                                                 'max_ndim': None, 'min_ndim': 2,
                                                                 'axes': {'-1': int(fan_in)}}},
            'build_input_shape': {'class_name': 'TensorShape', 'items': [None, int(fan_in)]}}


def _layer_units(V, d):
    """(units, activation) of every Dense layer by its attribute path (model.py:27-33, 58-64)."""
    out = {'encoder/encoded_1': (d, 'relu'), 'encoder/encoded_2': (256, 'relu'),
           'encoder/encoded_3': (128, 'relu'), 'encoder/bottleneck': (64, 'relu')}
    for pre, act in (('decoder', 'sigmoid'), ('decoder_for_reg', 'softmax')):
        out.update({f'{pre}/decoded_1': (128, 'relu'), f'{pre}/decoded_2': (256, 'relu'),
                    f'{pre}/decoded_3': (d, 'relu'), f'{pre}/reconstruct': (V, act)})
    return out


def _fan_in(path, V, d):
    return {'encoded_1': V, 'encoded_2': d, 'encoded_3': 256, 'bottleneck': 128, 'decoded_1': 64,
            'decoded_2': 128, 'decoded_3': 256, 'reconstruct': d}[path.split('/')[1]]


def _model_meta(V, d, reg, lr, beta1, beta2):
    opt = {'class_name': 'Adam', 'config': {'name': 'Adam', 'learning_rate': lr, 'decay': 0.0, 'beta_1': beta1,
                                            'beta_2': beta2, 'epsilon': 1e-07, 'amsgrad': False}}
    return {'class_name': 'CC_Recommender', 'name': 'cc__recommender', 'trainable': True,
            'expects_training_arg': True, 'dtype': 'float32', 'batch_input_shape': None,
            'must_restore_from_config': False, 'is_graph_network': False,
            'save_spec': [[{'class_name': 'TypeSpec', 'type_spec': 'tf.TensorSpec',
                            'serialized': [[None, int(V)], 'float32', 'input_1']}] * 2],
            'keras_version': None, 'backend': 'tensorflow', 'model_config': {'class_name': 'CC_Recommender'},
            'training_config': {'loss': ['binary_crossentropy', 'kullback_leibler_divergence'],
                                'metrics': ['accuracy'], 'weighted_metrics': None,
                                'loss_weights': [1.0, float(reg)], 'optimizer_config': opt}}


def _tensor_shape(shape):
    return b''.join(_field(2, 2, _field(1, 0, int(s))) for s in shape)


def _user_object(identifier, metadata=None):
    body = _field(1, 2, identifier.encode()) + _field(2, 2, _field(1, 0, 1) + _field(2, 0, 1))
    if metadata is not None:
        body += _field(3, 2, json.dumps(metadata, separators=(', ', ': ')).encode())
    return body


def _variable(dtype, shape, trainable, sync, agg, name):
    body = _field(1, 0, dtype) + _field(2, 2, _tensor_shape(shape))
    if trainable:
        body += _field(3, 0, 1)
    if sync:
        body += _field(4, 0, sync)
    if agg:
        body += _field(5, 0, agg)
    return body + _field(6, 2, name.encode())


def saved_object_graph(tensors, V, d, reg=0.0, lr=1e-3, beta1=0.9, beta2=0.999):
    """SavedObjectGraph bytes mirroring tensors[OBJECT_GRAPH_KEY] node for node."""
    nodes = parse_object_graph(tensors[OBJECT_GRAPH_KEY])
    paths = {0: ''}
    for i, nd in enumerate(nodes):            # parents precede children in the object graph
        for c, local in nd['children']:
            paths.setdefault(c, (paths[i] + '/' + local).lstrip('/'))
    slot_nodes = {sv for nd in nodes for _, _, sv in nd['slots']}
    units = _layer_units(V, d)
    out = b''
    for i, nd in enumerate(nodes):
        body = b''.join(_field(1, 2, _field(1, 0, c) + _field(2, 2, l.encode())) for c, l in nd['children'])
        body += b''.join(_field(3, 2, _field(1, 0, o) + _field(2, 2, s.encode()) + _field(3, 0, sv))
                         for o, s, sv in nd['slots'])
        path = paths.get(i, '')
        if nd['attrs']:                          # a variable: its tensor in the bundle
            _, full, key = nd['attrs'][0]
            a = tensors[key]
            dt = DT_INT64 if a.dtype.kind == 'i' else DT_FLOAT
            if i in slot_nodes or path.startswith('optimizer/'):
                kind = (False, SYNC_AUTO, AGG_ONLY_FIRST_REPLICA if path == 'optimizer/iter' else AGG_NONE)
            elif path.startswith('keras_api/'):
                kind = (False, SYNC_ON_READ, AGG_SUM)
            else:
                kind = (True, SYNC_AUTO, AGG_NONE)
            body += _field(7, 2, _variable(dt, a.shape, *kind, full))
        elif i == 0:
            body += _field(4, 2, _user_object('_tf_keras_model', _model_meta(V, d, reg, lr, beta1, beta2)))
        elif path in _SUBMODEL:
            cls, name = _SUBMODEL[path]
            body += _field(4, 2, _user_object('_tf_keras_model', {
                'class_name': cls, 'name': name, 'trainable': True, 'expects_training_arg': True,
                'dtype': 'float32', 'batch_input_shape': None, 'must_restore_from_config': False,
                'is_graph_network': False, 'model_config': {'class_name': cls}}))
        elif path in units:
            u, act = units[path]
            body += _field(4, 2, _user_object('_tf_keras_layer', _dense_meta(_LAYER_NAMES[path], u, act,
                                                                             _fan_in(path, V, d))))
        elif path == 'optimizer':
            body += _field(4, 2, _user_object('_generic_user_object'))
        elif path == 'keras_api' or path == 'keras_api/metrics':
            body += _field(4, 2, _user_object('_generic_user_object' if path == 'keras_api'
                                              else 'trackable_list_wrapper'))
        elif path.startswith('keras_api/metrics/'):
            name = {'0': 'loss', '1': 'output_1_loss'}.get(path.rsplit('/', 1)[1], 'mean')
            body += _field(4, 2, _user_object('_tf_keras_metric', {
                'class_name': 'Mean', 'name': name, 'dtype': 'float32',
                'config': {'name': name, 'dtype': 'float32'}}))
        else:
            body += _field(4, 2, _user_object('_generic_user_object'))
        out += _field(1, 2, body)
    return out


def saved_model_proto(tensors, V, d, **kw):
    """SavedModel bytes: schema version 1, one MetaGraphDef {MetaInfoDef tags ["serve"], an empty
    GraphDef with its version, a V2 SaverDef, the SavedObjectGraph}."""
    meta_info = _field(1, 2, PRODUCER.encode()) + _field(4, 2, b'serve')
    graph_def = _field(4, 2, _field(1, 0, 716))                  # versions {producer}
    saver = (_field(1, 2, b'saver_filename:0') + _field(2, 2, b'StatefulPartitionedCall_1:0')
             + _field(3, 2, b'StatefulPartitionedCall_2') + _field(5, 0, 1) + _field(7, 0, 2))
    mg = (_field(1, 2, meta_info) + _field(2, 2, graph_def) + _field(3, 2, saver)
          + _field(7, 2, saved_object_graph(tensors, V, d, **kw)))
    return _field(1, 0, SCHEMA_VERSION) + _field(2, 2, mg)


def parse_saved_model(b):
    """-> {'schema_version', 'tags', 'nodes': [{'children', 'slots', 'kind', ...}]}."""
    top = _parse(b)
    mg = _parse(top[2][0])
    info = _parse(mg.get(1, [b''])[0])
    og = _parse(mg[7][0])
    nodes = []
    for body in og.get(1, []):
        f = _parse(body)
        nd = {'children': [(_parse(c).get(1, [0])[0], _parse(c).get(2, [b''])[0].decode()) for c in f.get(1, [])],
              'slots': [(_parse(x).get(1, [0])[0], _parse(x).get(2, [b''])[0].decode(), _parse(x).get(3, [0])[0])
                        for x in f.get(3, [])]}
        if 7 in f:
            v = _parse(f[7][0])
            nd.update(kind='variable', dtype=v.get(1, [0])[0], trainable=bool(v.get(3, [0])[0]),
                      shape=[_parse(dim).get(1, [0])[0] for dim in _parse(v.get(2, [b''])[0]).get(2, [])],
                      name=v.get(6, [b''])[0].decode(), synchronization=v.get(4, [0])[0],
                      aggregation=v.get(5, [0])[0])
        elif 4 in f:
            u = _parse(f[4][0])
            nd.update(kind='user_object', identifier=u.get(1, [b''])[0].decode(),
                      metadata=json.loads(u[3][0].decode()) if 3 in u else None)
        nodes.append(nd)
    return {'schema_version': top.get(1, [0])[0], 'tags': [t.decode() for t in info.get(4, [])],
            'producer': info.get(1, [b''])[0].decode(), 'nodes': nodes}

