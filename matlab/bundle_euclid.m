function [K_, Te_, w_, Xe_, error_] = bundle_euclid(K, Te, w, Xe, x, varargin)
%BUNDLE_EUCLID  Euclidean bundle adjustment on an AMD MI355X (vlgba drop-in).
%
%   [K_ Te_ w_ Xe_ error_] = bundle_euclid(K, Te, w, Xe, x, ...)
%
%   Same signature, options and outputs as VLG's toolbox/bundle/bundle_euclid.m:
%     K (4xm) fx fy cx cy, Te (3xm), w (3xm) Rodrigues vectors, Xe (4xn)
%     homogeneous points (Xe(4,:) passed through), x (3xnxm) image points.
%   Options: 'fix_structure', 'fix_motion', 'fix_pivot' pivot (a logical mask
%   or camera numbers, as U(:,:,pivot) indexes in VLG's bundle_euclid.m),
%   'fix_calibration', 'fix_principal', 'visibility' V (nxm), 'verbose'.
%   error_ is the SSE / sum(visibility) before the first and after every
%   accepted step.
%
%   The whole Levenberg-Marquardt loop runs in one call of the fused MEX
%   gateway mex_bundle_euclid_lm (libvlgba: HIP kernels for gfx950); put this
%   directory before toolbox/bundle on the MATLAB path.  The staged gateways
%   mex_bundle_1_XABeUVWeAeB / mex_bundle_2_Se_ / mex_bundle_3_db_new of this
%   directory serve the reference's own bundle_euclid.m unchanged.
%
%   Extra options of this build: 'semantics', 'nomex' (the arithmetic of
%   bundle_euclid_nomex.m), 'max_iter', N, 'stop_rel', r (the 1e-3 of the
%   stop rule), 'device', D, 'ordered' (sequential sums), 'parity' (ordered
%   sums + sequential solve: the trajectory of the CPU oracle bit for bit).

if nargin < 5
    help bundle_euclid
    return;
end
m = size(w, 2);
n = size(x, 2);

opts = struct('fix_structure', 0, 'fix_motion', 0, 'verbose', 0, 'pivot', [], 'pivot_mask', [], ...
              'semantics', 0, 'max_iter', 0, 'stop_rel', 0, 'device', 0, 'ordered', 0);
nvk = 4;                                    % free fx fy cx cy
vis = [];
k = 1;
while k <= numel(varargin)
    name = lower(varargin{k});
    if strcmp(name, 'fix_structure'),      opts.fix_structure = 1;
    elseif strcmp(name, 'fix_motion'),     opts.fix_motion = 1;
    elseif strcmp(name, 'fix_pivot')
        pv = varargin{k+1}; k = k + 1;      % mask or index list (bundle_euclid.m:150-153)
        if islogical(pv), opts.pivot_mask = double(pv(:)');
        else,             opts.pivot = double(pv(:)'); end
    elseif strcmp(name, 'fix_calibration'), nvk = 0;
    elseif strcmp(name, 'fix_principal'),  nvk = 1;
    elseif strcmp(name, 'visibility'),     vis = varargin{k+1}; k = k + 1;
    elseif strcmp(name, 'verbose'),        opts.verbose = 1;
    elseif strcmp(name, 'semantics'),      opts.semantics = double(strcmpi(varargin{k+1}, 'nomex')); k = k + 1;
    elseif strcmp(name, 'max_iter'),       opts.max_iter = varargin{k+1}; k = k + 1;
    elseif strcmp(name, 'device'),         opts.device = varargin{k+1}; k = k + 1;
    elseif strcmp(name, 'stop_rel'),       opts.stop_rel = varargin{k+1}; k = k + 1;
    elseif strcmp(name, 'ordered'),        opts.ordered = 1;
    elseif strcmp(name, 'parity'),         opts.ordered = 2;
    end                                     % unknown names are ignored, as in VLG
    k = k + 1;
end
if isempty(vis)
    vis = reshape(x(1,:,:) ~= 0 | x(2,:,:) ~= 0, n, m);
end
if opts.semantics
    opts.pivot = [];                        % bundle_euclid_nomex has no fix_pivot
    opts.pivot_mask = [];
end

% parameters as VLG packs them: a = [w; T; (fx) | (fx fy cx cy)], b = Xe(1:3,:)
switch nvk
    case 0, a = [w; Te];
    case 1, a = [w; Te; K(1,:)];
    otherwise, a = [w; Te; K];
end
[a, b, error_] = mex_bundle_euclid_lm(double(K), double(a), double(Xe(1:3,:)), ...
                                      double(x(1:2,:,:)), double(vis), opts);

K_ = K;
if nvk == 1
    K_(1:2,:) = [a(7,:); a(7,:)];
elseif nvk == 4
    K_ = a(7:10,:);
end
w_ = a(1:3,:);
Te_ = a(4:6,:);
if opts.semantics
    Xe_ = [b; ones(1, n)];
else
    Xe_ = [b; Xe(4,:)];
end
end
